// In-kernel phase timing of one LDS-DMA GEMM config (diagnostic executable): compiles
// csrc/kernels/gemm_glds_impl.h (configs 34, 24, 27, 17, 25, 22) into this translation unit with DLS_STAMP recording
// s_memrealtime (100 MHz) per workgroup at: tile start, after the main loop, after the output
// image is in LDS, after the store pass.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/kernels benchmarks/gemm_stamps.hip -o gpubin/gemm_stamps
//   gpubin/gemm_stamps <cfg> <M> <N> <K>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ unsigned long long g_stamps[4096 * 4];
#define DLS_STAMP(k)                                                                     \
  if (threadIdx.x == 0 && blockIdx.x < 4096) {                                           \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                          \
    g_stamps[blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memrealtime();                   \
  }
#include "../csrc/kernels/gemm_glds_impl.h"
DLS_GLDS_DEFINE(34)
DLS_GLDS_DEFINE(24)
DLS_GLDS_DEFINE(27)
DLS_GLDS_DEFINE(17)
DLS_GLDS_DEFINE(25)
DLS_GLDS_DEFINE(22)
// splitk = 1 only: the split-K reduce launcher of the library is stubbed out below
static bool launch_gemm_glds_local(const GemmArgs& a, int cfg, int splitk) {
  switch (cfg) {
    case 24: return glds_launch_cfg24(a, splitk, nullptr, 0, nullptr, 0, 1e-5f, nullptr, false);
    case 27: return glds_launch_cfg27(a, splitk, nullptr, 0, nullptr, 0, 1e-5f, nullptr, false);
    case 17: return glds_launch_cfg17(a, splitk, nullptr, 0, nullptr, 0, 1e-5f, nullptr, false);
    case 25: return glds_launch_cfg25(a, splitk, nullptr, 0, nullptr, 0, 1e-5f, nullptr, false);
    case 22: return glds_launch_cfg22(a, splitk, nullptr, 0, nullptr, 0, 1e-5f, nullptr, false);
    default: return glds_launch_cfg34(a, splitk, nullptr, 0, nullptr, 0, 1e-5f, nullptr, false);
  }
}
bool glds_reduce(const GemmArgs&, int, float*, hipStream_t, const float*, int, float, const int*, const Epi&) { return false; }

int main(int argc, char** argv) {
  const int cfg = argc > 1 ? atoi(argv[1]) : 34;
  const int M = argc > 2 ? atoi(argv[2]) : 512, N = argc > 3 ? atoi(argv[3]) : 32768, K = argc > 4 ? atoi(argv[4]) : 768;
  std::vector<unsigned short> h((size_t)std::max(M, N) * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (unsigned short)(rand() & 0x3ff);  // bf16 in [1, 2)
  void *A, *W, *C;
  hipMalloc(&A, (size_t)M * K * 2);
  hipMalloc(&W, (size_t)N * K * 2);
  hipMalloc(&C, (size_t)M * N * 2);
  hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice);
  hipMemcpy(W, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice);
  GemmArgs g{};
  g.A = A; g.lda = K; g.W = W; g.ldw = K; g.C = C; g.ldc = N; g.M = M; g.N = N; g.K = K; g.alpha = 1.f;
  g.config = cfg;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipMemset(C, 0, (size_t)M * N * 2);
  for (int i = 0; i < 5; ++i) launch_gemm_glds_local(g, cfg, 1);
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), std::vector<unsigned long long>(4096 * 4, 0).data(), 4096 * 4 * 8);
  hipEventRecord(e0);
  launch_gemm_glds_local(g, cfg, 1);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(4096 * 4);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8);
  int nb = 0;
  for (int b = 0; b < 4096; ++b)
    if (st[b * 4]) nb = b + 1;
  unsigned long long t0 = ~0ull, tend = 0;
  std::vector<double> d01, d12, d23, start, end;
  for (int b = 0; b < nb; ++b) {
    const unsigned long long* s = &st[b * 4];
    if (!s[0]) continue;
    t0 = std::min(t0, s[0]);
    tend = std::max(tend, s[3]);
  }
  for (int b = 0; b < nb; ++b) {
    const unsigned long long* s = &st[b * 4];
    if (!s[0]) continue;
    d01.push_back((s[1] - s[0]) * 0.01);
    d12.push_back((s[2] - s[1]) * 0.01);
    d23.push_back((s[3] - s[2]) * 0.01);
    start.push_back((s[0] - t0) * 0.01);
    end.push_back((s[3] - t0) * 0.01);
  }
  auto q = [](std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[(size_t)(p * (v.size() - 1))];
  };
  printf("cfg %d  M %d N %d K %d: event %.2f us; blocks %zu; first-start -> last-end %.2f us\n", cfg, M, N, K,
         ms * 1e3, d01.size(), (tend - t0) * 0.01);
  printf("  start offset   min %.2f med %.2f max %.2f us\n", q(start, 0), q(start, .5), q(start, 1));
  printf("  main loop      min %.2f med %.2f max %.2f us\n", q(d01, 0), q(d01, .5), q(d01, 1));
  printf("  image to LDS   min %.2f med %.2f max %.2f us\n", q(d12, 0), q(d12, .5), q(d12, 1));
  printf("  store pass     min %.2f med %.2f max %.2f us\n", q(d23, 0), q(d23, .5), q(d23, 1));
  printf("  end offset     min %.2f med %.2f max %.2f us\n", q(end, 0), q(end, .5), q(end, 1));
  return 0;
}
