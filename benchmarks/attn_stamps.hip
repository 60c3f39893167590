// In-kernel phase timing of the flash-attention kernel (diagnostic executable): compiles
// csrc/kernels/attention.hip into this translation unit with DLS_ASTAMP reading s_memrealtime
// (100 MHz) into registers of every block's first thread at: block start, first K/V tile
// landed, key loop done, key-split merge done, output stored; they are written out once at the
// end of the block. GPT-2 shape: S 512, 12 heads x 64, causal, batch 1.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/kernels benchmarks/attn_stamps.hip -o gpubin/attn_stamps
//   gpubin/attn_stamps [variant] [S] [heads] [flags]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ unsigned long long g_astamps[4096 * 5];
#define DLS_ASTAMP_DECL() unsigned long long ts_[5] = {0, 0, 0, 0, 0};
#define DLS_ASTAMP(k) ts_[k] = __builtin_amdgcn_s_memrealtime();
#define DLS_ASTAMP_STORE()                                                                           \
  if (threadIdx.x == 0) {                                                                            \
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                  \
    if (lin < 4096) {                                                                                \
      g_astamps[lin * 5 + 0] = ts_[0];                                                                  \
      g_astamps[lin * 5 + 1] = ts_[1];                                                                  \
      g_astamps[lin * 5 + 2] = ts_[2];                                                                  \
      g_astamps[lin * 5 + 3] = ts_[3];                                                                  \
      g_astamps[lin * 5 + 4] = ts_[4];                                                                  \
    }                                                                                                \
  }
#include "../csrc/kernels/attention.hip"

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 0;
  const int S = argc > 2 ? atoi(argv[2]) : 512, H = argc > 3 ? atoi(argv[3]) : 12, D = 64;
  const int flags = argc > 4 ? atoi(argv[4]) : 0;
  std::vector<unsigned short> h((size_t)S * 3 * H * D);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (unsigned short)(rand() & 0x3ff);
  void *qkv, *o;
  hipMalloc(&qkv, h.size() * 2);
  hipMalloc(&o, (size_t)S * H * D * 2);
  hipMemcpy(qkv, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  const char* base = static_cast<const char*>(qkv);
  AttnArgs a{base, 3 * H * D, base + H * D * 2, 3 * H * D, base + 2 * H * D * 2, 3 * H * D, o, H * D,
             1, S, H, H, D, 0.125f, 1, variant, 0, 0, flags, nullptr, nullptr};
  if (variant == 14) {  // split variant: partials + zeroed tickets
    size_t pf = 0, nc = 0;
    attention_split_sizes(a, &pf, &nc);
    hipMalloc(&a.part, pf * 4);
    hipMalloc(&a.cnt, nc * 4);
    hipMemset(a.cnt, 0, nc * 4);
  }
  for (int i = 0; i < 5; ++i) launch_attention_fwd(a, 0);
  hipDeviceSynchronize();
  hipMemcpyToSymbol(HIP_SYMBOL(g_astamps), std::vector<unsigned long long>(4096 * 5, 0).data(), 4096 * 5 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  launch_attention_fwd(a, 0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(4096 * 5);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_astamps), st.size() * 8);
  unsigned long long t0 = ~0ull, tend = 0;
  int nb = 0;
  for (int b = 0; b < 4096; ++b)
    if (st[b * 5]) {
      t0 = std::min(t0, st[b * 5]);
      tend = std::max(tend, st[b * 5 + 4]);
      ++nb;
    }
  printf("flags %d ", flags);
  printf("variant %d S %d heads %d: event %.2f us; blocks %d; first-start -> last-end %.2f us\n", variant, S, H,
         ms * 1e3, nb, (tend - t0) * 0.01);
  const char* names[] = {"start offset", "first K/V tile", "key loop", "merge", "normalise+store"};
  for (int k = 0; k < 5; ++k) {
    std::vector<double> v;
    for (int b = 0; b < 4096; ++b)
      if (st[b * 5]) v.push_back(k == 0 ? (st[b * 5] - t0) * 0.01 : (st[b * 5 + k] - st[b * 5 + k - 1]) * 0.01);
    std::sort(v.begin(), v.end());
    printf("  %-16s min %.2f med %.2f max %.2f us\n", names[k], v.front(), v[v.size() / 2], v.back());
  }
  // the heaviest blocks (last query tile of each head: blockIdx.x = 0 under heaviest-first)
  std::vector<double> heavy;
  for (int b = 0; b < 4096; ++b)
    if (st[b * 5] && (b % ((S + 31) / 32)) == 0) heavy.push_back((st[b * 5 + 4] - st[b * 5]) * 0.01);
  if (!heavy.empty()) {
    std::sort(heavy.begin(), heavy.end());
    printf("  heaviest blocks  start->end med %.2f max %.2f us\n", heavy[heavy.size() / 2], heavy.back());
  }
  return 0;
}
