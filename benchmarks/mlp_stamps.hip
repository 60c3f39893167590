// Where the one-launch GPT-2 MLP block's time goes: in-kernel s_memrealtime
// stamps (100 MHz) per workgroup of csrc/kernels/gemm_fused.hip, compiled into this diagnostic
// executable, and event times of
//   unfused   fc1 (folded LN + GELU, config 25) then fc2 (+ residual, config 45): two launches
//   fused     mlp_fused_kernel<false>: one launch, fc2 polls fc1's row-block arrivals
//   prefetch  mlp_fused_kernel<true>: each workgroup DMAs its share of its fc2 weight panel
//             into the idle LDS before the poll (the panel lands in its XCD's L2)
// Per-block phases of one fused launch: phase 1 (fc1 tile + publish), the wait (poll, and the
// prefetch), phase 2 (fc2 tile: main loop, LDS image, store pass).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -Icsrc/kernels \
//         benchmarks/mlp_stamps.hip -o gpubin/mlp_stamps
//   gpubin/mlp_stamps [iters]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__device__ unsigned long long g_stamps[256 * 8];
#define DLS_STAMP(k)                                                   \
  if (threadIdx.x == 0 && blockIdx.x < 256) {                          \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");        \
    g_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  }
#include "../csrc/kernels/gemm_fused.hip"
DLS_GLDS_DEFINE(25)
DLS_GLDS_DEFINE(45)
bool glds_reduce(const GemmArgs&, int, float*, hipStream_t, const float*, int, float, const int*, const Epi&) {
  return false;
}

static void fill(void* p, size_t n, float scale, unsigned seed) {
  std::vector<unsigned short> h(n);
  srand(seed);
  for (size_t i = 0; i < n; ++i) {
    const float v = scale * ((rand() & 0xffff) / 32768.f - 1.f);
    unsigned u;
    memcpy(&u, &v, 4);
    h[i] = (unsigned short)(u >> 16);
  }
  hipMemcpy(p, h.data(), n * 2, hipMemcpyHostToDevice);
}

static double q(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  const int M = 512, H = 768, F = 3072, Hout = 768;
  void *x, *w1, *b1, *h, *w2, *b2, *r, *o;
  float *colsum, *ext;
  int* sync;
  hipMalloc(&x, (size_t)M * H * 2);
  hipMalloc(&w1, (size_t)F * H * 2);
  hipMalloc(&b1, (size_t)F * 2);
  hipMalloc(&h, (size_t)M * F * 2);
  hipMalloc(&w2, (size_t)Hout * F * 2);
  hipMalloc(&b2, (size_t)Hout * 2);
  hipMalloc(&r, (size_t)M * Hout * 2);
  hipMalloc(&o, (size_t)M * Hout * 2);
  hipMalloc(&colsum, (size_t)F * 4);
  hipMalloc(&ext, (size_t)M * 2 * 4);
  hipMalloc(&sync, 64 * 4);
  fill(x, (size_t)M * H, 1.f, 1);
  fill(w1, (size_t)F * H, 0.05f, 2);
  fill(b1, F, 0.1f, 3);
  fill(w2, (size_t)Hout * F, 0.05f, 4);
  fill(b2, Hout, 0.1f, 5);
  fill(r, (size_t)M * Hout, 1.f, 6);
  hipMemset(colsum, 0, (size_t)F * 4);
  std::vector<float> st2(M * 2);
  for (int m = 0; m < M; ++m) {
    st2[2 * m] = 0.f;
    st2[2 * m + 1] = (float)H;  // mean 0, variance 1
  }
  hipMemcpy(ext, st2.data(), st2.size() * 4, hipMemcpyHostToDevice);
  hipMemset(sync, 0, 64 * 4);

  GemmArgs g1{};
  g1.A = x; g1.lda = H; g1.W = w1; g1.ldw = H; g1.C = h; g1.ldc = F; g1.bias = b1;
  g1.M = M; g1.N = F; g1.K = H; g1.act = ACT_GELU_TANH; g1.alpha = 1.f; g1.ext_stats = ext;
  GemmArgs g2{};
  g2.A = h; g2.lda = F; g2.W = w2; g2.ldw = F; g2.C = o; g2.ldc = Hout; g2.bias = b2; g2.R = r; g2.ldr = Hout;
  g2.M = M; g2.N = Hout; g2.K = F; g2.act = 0; g2.alpha = 1.f;
  MlpFusedArgs p{x, H, w1, H, b1, colsum, ext, 1, 1e-5f, ACT_GELU_TANH, h, F, w2, F, b2, r, Hout, o, Hout,
                 nullptr, M, H, F, Hout, sync, sync + M / 64, sync + 2 * (M / 64), 1 << 22};
  if (!mlp_fused_supported(M, H, F, Hout, 256)) {
    printf("shape not supported\n");
    return 1;
  }
  auto unfused = [&] {
    glds_launch_cfg25(g1, 1, nullptr, 0, colsum, 1, 1e-5f, nullptr, false);
    glds_launch_cfg45(g2, 1, nullptr, 0, nullptr, 0, 1e-5f, nullptr, false);
  };
  auto fused = [&](int pre) {
    p.prefetch_w2 = pre;
    launch_mlp_fused(p, 0);
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](auto fn) {
    for (int i = 0; i < 20; ++i) fn();
    hipEventRecord(e0);
    for (int i = 0; i < iters; ++i) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3 / iters;
  };
  // alternate the three variants, three rounds each (same box, same state)
  double tu = 0, tf = 0, tp = 0;
  for (int rep = 0; rep < 3; ++rep) {
    const double a = timeit(unfused), b = timeit([&] { fused(0); }), c = timeit([&] { fused(1); });
    printf("round %d: unfused %.2f us  fused %.2f us  fused+prefetch %.2f us per MLP block\n", rep, a, b, c);
    tu += a / 3;
    tf += b / 3;
    tp += c / 3;
  }
  int err = 0;
  hipMemcpy(&err, sync + 2 * (M / 64), 4, hipMemcpyDeviceToHost);
  printf("mean: unfused %.2f  fused %.2f  fused+prefetch %.2f us  (poll error word %d)\n", tu, tf, tp, err);
  for (int pre = 0; pre < 2; ++pre) {
    hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), std::vector<unsigned long long>(256 * 8, 0).data(), 256 * 8 * 8);
    fused(pre);
    hipDeviceSynchronize();
    std::vector<unsigned long long> s(256 * 8);
    hipMemcpyFromSymbol(s.data(), HIP_SYMBOL(g_stamps), s.size() * 8);
    unsigned long long t0 = ~0ull, tend = 0;
    for (int b = 0; b < 256; ++b) {
      t0 = std::min(t0, s[b * 8 + 4]);
      tend = std::max(tend, s[b * 8 + 3]);
    }
    std::vector<double> st, p1, wt, mloop, img, store, pub;
    for (int b = 0; b < 256; ++b) {
      const unsigned long long* v = &s[b * 8];
      st.push_back((v[4] - t0) * 0.01);
      p1.push_back((v[5] - v[4]) * 0.01);
      pub.push_back((v[5] - t0) * 0.01);
      wt.push_back((v[6] - v[5]) * 0.01);
      mloop.push_back((v[1] - v[0]) * 0.01);
      img.push_back((v[2] - v[1]) * 0.01);
      store.push_back((v[3] - v[2]) * 0.01);
    }
    printf("fused%s: first start -> last end %.2f us (256 blocks)\n", pre ? "+prefetch" : "", (tend - t0) * 0.01);
    auto row = [](const char* n, const std::vector<double>& v) {
      printf("  %-28s min %6.2f med %6.2f max %6.2f us\n", n, q(v, 0), q(v, .5), q(v, 1));
    };
    row("start offset", st);
    row("phase 1 (fc1 tile+publish)", p1);
    row("published at", pub);
    row(pre ? "wait (prefetch + poll)" : "wait (poll)", wt);
    row("phase 2 main loop", mloop);
    row("phase 2 image to LDS", img);
    row("phase 2 store pass", store);
  }
  return 0;
}
