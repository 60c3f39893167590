// Memory-bound element-wise kernels: GELU(tanh), residual add, SwiGLU, token+position
// embedding gather, rotary embedding. All move 16-byte (8 x bf16) vectors per lane and
// grid-stride over at most 256 CUs x 8 blocks (cdna_hip_programming.md Guideline 11,13).
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

inline int grid_for(int64_t n_vec) {
  int64_t g = (n_vec + 255) / 256;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

__global__ __launch_bounds__(256) void gelu_kernel(const bf16x8* __restrict__ x, bf16x8* __restrict__ y,
                                                   int64_t nvec) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const bf16x8 a = x[i];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(gelu_tanh(bf2f(a[e])));
    y[i] = o;
  }
}

__global__ __launch_bounds__(256) void add_kernel(const bf16x8* __restrict__ a, const bf16x8* __restrict__ b,
                                                  bf16x8* __restrict__ y, int64_t nvec) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const bf16x8 u = a[i], v = b[i];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(u[e]) + bf2f(v[e]));
    y[i] = o;
  }
}

// gu [M][2F] = [gate | up] -> y [M][F] = silu(gate) * up
__global__ __launch_bounds__(256) void swiglu_kernel(const bf16* __restrict__ gu, bf16* __restrict__ y, int M,
                                                     int F) {
  const int fv = F / 8;
  const int64_t nvec = (int64_t)M * fv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / fv, c = i % fv;
    const bf16x8 g = reinterpret_cast<const bf16x8*>(gu + m * 2 * F)[c];
    const bf16x8 u = reinterpret_cast<const bf16x8*>(gu + m * 2 * F + F)[c];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(silu(bf2f(g[e])) * bf2f(u[e]));
    reinterpret_cast<bf16x8*>(y + m * F)[c] = o;
  }
}

// y[m] = wte[tok[m]] + wpe[m % S] (wpe may be null: token embedding only)
// zbuf (optional): fp32 words zeroed on the way (the step's row-statistics accumulators, so the
// first node of the step clears them instead of a separate fill kernel)
__global__ __launch_bounds__(256) void embedding_kernel(const int32_t* __restrict__ tok,
                                                        const bf16* __restrict__ wte,
                                                        const bf16* __restrict__ wpe, bf16* __restrict__ y, int M,
                                                        int S, int H, float* __restrict__ zbuf, int zn,
                                                        float* __restrict__ stats) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < zn; i += gridDim.x * 256) zbuf[i] = 0.f;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int t = tok[row];
  const bf16x8* er = reinterpret_cast<const bf16x8*>(wte + (size_t)t * H);
  const bf16x8* pr = wpe ? reinterpret_cast<const bf16x8*>(wpe + (size_t)(row % S) * H) : nullptr;
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + (size_t)row * H);
  float s1 = 0.f, s2 = 0.f;
  for (int c = lane; c < H / 8; c += 64) {
    bf16x8 a = er[c];
    if (pr) {
      const bf16x8 p = pr[c];
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = f2bf(bf2f(a[e]) + bf2f(p[e]));
    }
    yr[c] = a;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = bf2f(a[e]);
      s1 += v;
      s2 += v * v;
    }
  }
  // the row's (sum, sum of squares) for the next folded norm (the wave owns the row: plain
  // stores into a region the zeroing above does not cover)
  if (stats) {
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      stats[2 * row] = s1;
      stats[2 * row + 1] = s2;
    }
  }
}

// Rotary embedding (rotate-half convention), in place on the q heads (columns
// [0, n_head*D)) and k heads (columns [k_col, k_col + n_kv*D)) of each token row.
// cos/sin tables [S][D/2] fp32 are precomputed on the host (no on-device trig).
// RoPE (rotate-half) in place on the q and k column ranges of the fused qkv activation:
// one thread per (token, head, 8 consecutive rotary pairs) -> 16-B loads of both halves and
// 32-B loads of the cos/sin rows (tables are [S][D/2] fp32).
__global__ __launch_bounds__(256) void rope_kernel(bf16* __restrict__ qkv, int ld, int M, int S, int n_head,
                                                   int n_kv, int D, int k_col, const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t) {
  const int half = D / 2, hv = half / 8;
  const int heads = n_head + n_kv;
  const int64_t total = (int64_t)M * heads * hv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int j = (int)(i % hv) * 8;
    const int64_t t = i / hv;
    const int hh = (int)(t % heads);
    const int m = (int)(t / heads);
    const int pos = m % S;
    const int col = hh < n_head ? hh * D : k_col + (hh - n_head) * D;
    bf16* base = qkv + (size_t)m * ld + col;
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(base + j);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(base + j + half);
    const f32x4* cp = reinterpret_cast<const f32x4*>(cos_t + (size_t)pos * half + j);
    const f32x4* sp = reinterpret_cast<const f32x4*>(sin_t + (size_t)pos * half + j);
    const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
    bf16x8 oa, ob;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float c = e < 4 ? c0[e] : c1[e - 4], sn = e < 4 ? s0[e] : s1[e - 4];
      const float x1 = bf2f(a[e]), x2 = bf2f(b[e]);
      oa[e] = f2bf(x1 * c - x2 * sn);
      ob[e] = f2bf(x2 * c + x1 * sn);
    }
    *reinterpret_cast<bf16x8*>(base + j) = oa;
    *reinterpret_cast<bf16x8*>(base + j + half) = ob;
  }
}

}  // namespace

void launch_gelu(const void* x, void* y, int64_t n, hipStream_t s) {
  const int64_t nv = n / 8;
  hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(nv)), dim3(256), 0, s, (const bf16x8*)x, (bf16x8*)y, nv);
}

void launch_add(const void* a, const void* b, void* y, int64_t n, hipStream_t s) {
  const int64_t nv = n / 8;
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(nv)), dim3(256), 0, s, (const bf16x8*)a, (const bf16x8*)b,
                     (bf16x8*)y, nv);
}

void launch_swiglu(const void* gu, void* y, int M, int F, hipStream_t s) {
  hipLaunchKernelGGL(swiglu_kernel, dim3(grid_for((int64_t)M * F / 8)), dim3(256), 0, s, (const bf16*)gu,
                     (bf16*)y, M, F);
}

void launch_embedding(const int32_t* tokens, const void* wte, const void* wpe, void* y, int M, int S, int H,
                      hipStream_t s, float* zbuf, int zn, float* stats) {
  hipLaunchKernelGGL(embedding_kernel, dim3((M + 3) / 4), dim3(256), 0, s, tokens, (const bf16*)wte,
                     (const bf16*)wpe, (bf16*)y, M, S, H, zbuf, zn, stats);
}

void launch_rope(void* qkv, int ld, int M, int S, int n_head, int n_kv_head, int D, int k_col, const float* cos_t,
                 const float* sin_t, hipStream_t s) {
  const int64_t total = (int64_t)M * (n_head + n_kv_head) * (D / 16);
  hipLaunchKernelGGL(rope_kernel, dim3(grid_for(total)), dim3(256), 0, s, (bf16*)qkv, ld, M, S, n_head,
                     n_kv_head, D, k_col, cos_t, sin_t);
}
