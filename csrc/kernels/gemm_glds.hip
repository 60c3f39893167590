// Multistage bf16 GEMM with LDS-DMA staging — host dispatch and the split-K reduce kernels.
// The device code and the per-config launcher live in gemm_glds_impl.h; every tile config is
// instantiated in one of the gemm_glds_cfg*.hip translation units (compiled in parallel).
#include <cstdlib>
#include "common.h"
#include "kernels.h"
#include "gemm_glds_cfgs.h"

namespace {
// Epilogue of a split-K GEMM for 8 consecutive columns c..c+7 of row m (non-SwiGLU):
// norm fold with handed-over row statistics, bias, activation, RoPE, residual.
struct ReduceNorm {
  const float* colsum;
  int mode;  // 0 none, 1 LayerNorm, 2 RMSNorm (statistics from ep.ext_stats)
  float eps;
  int K;
};

// (bv / rv: the bias and residual vectors, loaded by the caller — ahead of the partial slabs
// where it can, so the whole row costs one memory round trip)
__device__ __forceinline__ void reduce_finalize_pre(float (&x)[8], const float (&v)[8], int m, int c, bool has_bias,
                                                    const bf16x8& bv, bool has_r, const bf16x8& rv, int act,
                                                    float alpha, const Epi& ep, const ReduceNorm& nm) {
  float mu = 0.f, rs = 1.f;
  if (nm.mode != 0) {
    const float inv_k = 1.0f / (float)nm.K;
    const float a = ep.ext_stats[2 * m], q = ep.ext_stats[2 * m + 1];
    mu = nm.mode == 1 ? a * inv_k : 0.f;
    rs = rsqrtf(fmaxf(q * inv_k - mu * mu, 0.f) + nm.eps);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float z = nm.mode != 0 ? rs * (v[e] - mu * nm.colsum[c + e]) : alpha * v[e];
    x[e] = apply_act(z + (has_bias ? bf2f(bv[e]) : 0.f), act);
  }
  if (ep.rope.cols) rope_pairs<8>(x, m, c, ep.rope);
  if (has_r) {
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] += bf2f(rv[e]);
  }
}

__device__ __forceinline__ void reduce_finalize(float (&x)[8], const float (&v)[8], int m, int c,
                                                const bf16* __restrict__ bias, const bf16* __restrict__ R, int ldr,
                                                int act, float alpha, const Epi& ep, const ReduceNorm& nm) {
  bf16x8 bv = {}, rv = {};
  if (bias) bv = *reinterpret_cast<const bf16x8*>(bias + c);
  if (R) rv = *reinterpret_cast<const bf16x8*>(R + (size_t)m * ldr + c);
  reduce_finalize_pre(x, v, m, c, bias != nullptr, bv, R != nullptr, rv, act, alpha, ep, nm);
}

// out = act(alpha * sum_s P[s] + bias) + R, 8 columns per lane (N % 8 == 0). ACT_SWIGLU: P is in
// the interleaved W' space (N wide), out is N/2 wide: out col c <- gate 32(c/16) + c%16, up +16.
// rows (optional device int32[2]) restricts to a row range as in the GEMM.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ P, int splitk, int M, int N,
                                                            bf16* __restrict__ C, int ldc,
                                                            const bf16* __restrict__ bias,
                                                            const bf16* __restrict__ R, int ldr, int act,
                                                            float alpha, const int* __restrict__ rows,
                                                            int compact_rows, Epi ep, ReduceNorm nm) {
  const size_t slab = (size_t)M * N;
  int r0 = 0, nrows = M;
  if (rows != nullptr) {
    r0 = rows[0];
    nrows = rows[1] - r0;
    if (compact_rows) nrows = min(nrows, compact_rows);
  }
  const bool sw = act == ACT_SWIGLU;
  const int NO = sw ? N / 2 : N;
  const int nv = NO / 8;
  const int64_t total = (int64_t)nrows * nv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int m = r0 + (int)(i / nv), c = (int)(i % nv) * 8;
    const int pc = sw ? 32 * (c / 16) + (c % 16) : c;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0}, u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < splitk; ++s) {
      const f32x4* p = reinterpret_cast<const f32x4*>(P + s * slab + (size_t)m * N + pc);
      const f32x4 a = p[0], b = p[1];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += a[e];
        v[4 + e] += b[e];
      }
      if (sw) {
        const f32x4 a2 = p[4], b2 = p[5];  // +16 floats: the up half
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          u[e] += a2[e];
          u[4 + e] += b2[e];
        }
      }
    }
    bf16x8 o;
    if (sw) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = alpha * v[e] + (bias ? bf2f(bias[pc + e]) : 0.f);
        const float up = alpha * u[e] + (bias ? bf2f(bias[pc + 16 + e]) : 0.f);
        o[e] = f2bf(silu(g) * up);
      }
    } else {
      float x[8];
      reduce_finalize(x, v, m, c, bias, R, ldr, act, alpha, ep, nm);
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = f2bf(x[e]);
        const float y = bf2f(o[e]);
        s1 += y;
        s2 += y * y;
      }
      if (ep.stats_out) {
        // launched only when a wave's 64 consecutive items share one row (nv % 64 == 0 and
        // the loop stride is a multiple of 64): one pair of atomics per wave
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        if ((threadIdx.x & 63) == 0) {
          atomicAdd(ep.stats_out + 2 * m, s1);
          atomicAdd(ep.stats_out + 2 * m + 1, s2);
        }
      }
    }
    const size_t off = ((size_t)(compact_rows ? m - r0 : m) * ldc + c) * 2;
    if (ep.w_stream & 4) store16_pol<16>(C, off, *reinterpret_cast<const u32x4*>(&o));
    else store16_pol<0>(C, off, *reinterpret_cast<const u32x4*>(&o));
  }
}

// Row-per-wave reduce for a producer that must also emit its rows' statistics (sum, sum of
// squares of the rounded outputs) for the next folded norm: the wave owns the whole row, so
// the statistics are plain stores — no atomics.
__global__ __launch_bounds__(256) void splitk_reduce_rows_kernel(const float* __restrict__ P, int splitk, int M,
                                                                 int N, bf16* __restrict__ C, int ldc,
                                                                 const bf16* __restrict__ bias,
                                                                 const bf16* __restrict__ R, int ldr, int act,
                                                                 float alpha, Epi ep, ReduceNorm nm) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const size_t slab = (size_t)M * N;
  float s1 = 0.f, s2 = 0.f;
  for (int c = lane * 8; c < N; c += 512) {
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < splitk; ++s) {
      const f32x4* p = reinterpret_cast<const f32x4*>(P + s * slab + (size_t)m * N + c);
      const f32x4 a = p[0], b = p[1];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += a[e];
        v[4 + e] += b[e];
      }
    }
    float x[8];
    reduce_finalize(x, v, m, c, bias, R, ldr, act, alpha, ep, nm);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf(x[e]);
      const float y = bf2f(o[e]);
      s1 += y;
      s2 += y * y;
    }
    if (ep.w_stream & 4) store16_pol<16>(C, ((size_t)m * ldc + c) * 2, *reinterpret_cast<const u32x4*>(&o));
    else store16_pol<0>(C, ((size_t)m * ldc + c) * 2, *reinterpret_cast<const u32x4*>(&o));
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    ep.stats_out[2 * m] = s1;
    ep.stats_out[2 * m + 1] = s2;
  }
}

// Split-K reduce that ALSO normalises the rows for the next norm (the separate norm launch of
// a K > 1024 norm — Llama / Mixtral hidden 4096 — disappears): one workgroup owns a row, keeps
// its bf16-rounded outputs in registers, reduces their statistics across the workgroup and
// writes norm(row) * w (+ b) — the norm kernel's arithmetic on the same rounded inputs.
constexpr int RN_MAXV = 4;  // 8-column vectors per thread: N <= 256 * 8 * RN_MAXV
// VPT vectors per thread, SK split-K slices known at compile time (0: runtime count): every
// slab load of the row is issued before the first add (one memory round trip, not VPT x SK)
template <int VPT, int SK>
__global__ __launch_bounds__(256) void splitk_reduce_norm_kernel(const float* __restrict__ P, int splitk, int M,
                                                                 int N, bf16* __restrict__ C, int ldc,
                                                                 const bf16* __restrict__ bias,
                                                                 const bf16* __restrict__ R, int ldr, int act,
                                                                 float alpha, Epi ep, ReduceNorm nm,
                                                                 bf16* __restrict__ Y, int ldy,
                                                                 const bf16* __restrict__ nw,
                                                                 const bf16* __restrict__ nb, int nmode, float neps) {
  __shared__ float red[2][4];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t slab = (size_t)M * N;
  const int nsk = SK > 0 ? SK : splitk;
  // every other operand of the row is requested first, so it lands with the slabs
  bf16x8 rpre[VPT], bpre[VPT], wv[VPT], bv[VPT];
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const int cl = min((u * 256 + tid) * 8, N - 8);
    rpre[u] = R ? *reinterpret_cast<const bf16x8*>(R + (size_t)m * ldr + cl) : bf16x8{};
    bpre[u] = bias ? *reinterpret_cast<const bf16x8*>(bias + cl) : bf16x8{};
    wv[u] = *reinterpret_cast<const bf16x8*>(nw + cl);
    bv[u] = nb ? *reinterpret_cast<const bf16x8*>(nb + cl) : bf16x8{};
  }
  float v[VPT][8];
#pragma unroll
  for (int u = 0; u < VPT; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
  if constexpr (SK > 0) {
    f32x4 a[VPT][SK][2];
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const int cl = min((u * 256 + tid) * 8, N - 8);  // clamped, not guarded
#pragma unroll
      for (int s2 = 0; s2 < SK; ++s2) {
        const f32x4* p = reinterpret_cast<const f32x4*>(P + s2 * slab + (size_t)m * N + cl);
        a[u][s2][0] = p[0];
        a[u][s2][1] = p[1];
      }
    }
#pragma unroll
    for (int u = 0; u < VPT; ++u)
#pragma unroll
      for (int s2 = 0; s2 < SK; ++s2)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[u][e] += a[u][s2][0][e];
          v[u][e + 4] += a[u][s2][1][e];
        }
  } else {
    for (int s2 = 0; s2 < nsk; ++s2) {
#pragma unroll
      for (int u = 0; u < VPT; ++u) {
        const int cl = min((u * 256 + tid) * 8, N - 8);
        const f32x4* p = reinterpret_cast<const f32x4*>(P + s2 * slab + (size_t)m * N + cl);
        const f32x4 a0 = p[0], a1 = p[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[u][e] += a0[e];
          v[u][e + 4] += a1[e];
        }
      }
    }
  }
  float y[VPT][8];
  float s1 = 0.f;
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const int c = (u * 256 + tid) * 8;
    const int cl = min(c, N - 8);
    float x[8];
    reduce_finalize_pre(x, v[u], m, cl, bias != nullptr, bpre[u], R != nullptr, rpre[u], act, alpha, ep, nm);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf(x[e]);
      y[u][e] = c < N ? bf2f(o[e]) : 0.f;
      s1 += y[u][e];
    }
    if (c < N) {
      if (ep.w_stream & 4) store16_pol<16>(C, ((size_t)m * ldc + c) * 2, *reinterpret_cast<const u32x4*>(&o));
      else store16_pol<0>(C, ((size_t)m * ldc + c) * 2, *reinterpret_cast<const u32x4*>(&o));
    }
  }
  auto block_sum = [&](float t, int slot) {
    t = wave_sum(t);
    if (lane == 0) red[slot][wave] = t;
    __syncthreads();
    return red[slot][0] + red[slot][1] + red[slot][2] + red[slot][3];
  };
  const float inv_n = 1.0f / (float)N;
  float mean = 0.f;
  if (nmode == 1) mean = block_sum(s1, 0) * inv_n;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < VPT; ++u)
    if ((u * 256 + tid) * 8 < N)
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (y[u][e] - mean) * (y[u][e] - mean);
  const float rstd = rsqrtf(block_sum(q, 1) * inv_n + neps);
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const int c = (u * 256 + tid) * 8;
    if (c >= N) continue;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = (y[u][e] - mean) * rstd * bf2f(wv[u][e]);
      if (nb) t += bf2f(bv[u][e]);
      o[e] = f2bf(t);
    }
    if (ep.w_stream & 4) store16_pol<16>(Y, ((size_t)m * ldy + c) * 2, *reinterpret_cast<const u32x4*>(&o));
    else store16_pol<0>(Y, ((size_t)m * ldy + c) * 2, *reinterpret_cast<const u32x4*>(&o));
  }
}

}  // namespace

bool glds_reduce(const GemmArgs& a, int splitk, float* ws, hipStream_t s, const float* ln_colsum, int ln_mode,
                 float ln_eps, const int* rows, const Epi& ep) {
  {
    const ReduceNorm nm{ln_colsum, a.ext_stats ? ln_mode : 0, ln_eps, a.K};
    if (a.norm_out && !rows && a.act != kActSwiglu && a.N % 8 == 0 && a.N <= 256 * 8 * RN_MAXV) {
#define DLS_RN(VPT, SK)                                                                                          \
  hipLaunchKernelGGL((splitk_reduce_norm_kernel<VPT, SK>), dim3(a.M), dim3(256), 0, s, ws, splitk, a.M, a.N,        \
                     (bf16*)a.C, a.ldc, (const bf16*)a.bias, (const bf16*)a.R, a.ldr, a.act, a.alpha, ep, nm,     \
                     (bf16*)a.norm_out, a.ldn, (const bf16*)a.norm_w, (const bf16*)a.norm_b, a.norm_mode, a.norm_eps)
      if (a.N <= 256 * 8 * 2) {
        if (splitk == 2) DLS_RN(2, 2);
        else if (splitk == 4) DLS_RN(2, 4);
        else DLS_RN(2, 0);
      } else {
        if (splitk == 2) DLS_RN(4, 2);
        else if (splitk == 4) DLS_RN(4, 4);
        else DLS_RN(4, 0);
      }
#undef DLS_RN
      return true;
    }
    if (a.stats_out && !rows && a.act != kActSwiglu && (a.N / 8) % 64 != 0) {  // small rows: a wave per row
      hipLaunchKernelGGL(splitk_reduce_rows_kernel, dim3((a.M + 3) / 4), dim3(256), 0, s, ws, splitk, a.M, a.N,
                         (bf16*)a.C, a.ldc, (const bf16*)a.bias, (const bf16*)a.R, a.ldr, a.act, a.alpha, ep, nm);
    } else {
      const int64_t nvec = (int64_t)a.M * (a.N / 8);
      const int g = (int)std::min<int64_t>(2048, (nvec + 255) / 256);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g), dim3(256), 0, s, ws, splitk, a.M, a.N, (bf16*)a.C, a.ldc,
                         (const bf16*)a.bias, (const bf16*)a.R, a.ldr, a.act, a.alpha, rows, a.compact_rows, ep, nm);
    }
  }
  return false;
  return false;
}

namespace {

struct Shape {
  int bm, bn;
};
constexpr Shape kShapes[] = {{256, 128}, {128, 128}, {128, 64},  {64, 64},   {64, 128},  {64, 64},
                             {128, 64},  {128, 128}, {256, 256}, {256, 256}, {256, 128}, {128, 128},
                             {256, 256}, {256, 256}, {256, 128}, {128, 128}, {64, 64},   {64, 64},
                             {128, 64},  {64, 128},  {64, 64},   {64, 64},   {64, 96},   {32, 144},
                             {32, 48},   {64, 96},   {32, 144},  {32, 48},   {128, 128}, {192, 128},
                             {192, 128}, {192, 128}, {192, 128}, {192, 128}, {256, 256}, {256, 256},
                             {256, 224}, {256, 224}, {128, 96},  {128, 96},  {128, 64},  {192, 128},
                             {256, 144}, {256, 192}, {160, 256}, {32, 48},   {128, 128}, {128, 128}};
constexpr int kKStep[] = {64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64,
                          64, 64, 128, 128, 128, 128, 256, 256, 64, 64, 64, 128, 128, 128, 128,
                          64, 128, 64, 64, 64, 64, 64, 64, 64, 64, 128, 128, 64, 64, 64, 64, 256, 64, 64};
constexpr int kNumCfg = 48;
constexpr bool swiglu_bad(int c) { return (c >= 22 && c <= 27) || c == 36 || c == 38 || c == 39 || c == 42 || c == 45; }
static_assert(kNumCfg <= kGemmPersist, "config ids must stay below the persistent-launch flag");

using LaunchFn = bool (*)(const GemmArgs&, int, float*, hipStream_t, const float*, int, float, const int*, bool);
using GroupedFn = void (*)(const GemmArgs&, int, const int*, const unsigned long long*, const unsigned long long*,
                           hipStream_t, const int*);
#define DLS_GLDS_L(ID) glds_launch_cfg##ID,
#define DLS_GLDS_G(ID) glds_grouped_cfg##ID,
constexpr LaunchFn kLaunch[] = {DLS_GLDS_ALL(DLS_GLDS_L)};
constexpr GroupedFn kGrouped[] = {DLS_GLDS_ALL(DLS_GLDS_G)};
#undef DLS_GLDS_L
#undef DLS_GLDS_G
static_assert(sizeof(kLaunch) / sizeof(kLaunch[0]) == kNumCfg, "one launcher per config");

}  // namespace

int gemm_glds_num_configs() { return kNumCfg; }
int gemm_glds_kstep(int cfg) { return kKStep[(cfg & (kGemmPersist - 1)) < kNumCfg ? (cfg & (kGemmPersist - 1)) : 3]; }

// Heuristic: largest tile whose grid (times a split-K factor that keeps >= 4 K-tiles per
// block) reaches ~256 blocks; split-K only when the output grid alone is too small.
void gemm_glds_pick(int M, int N, int K, int* cfg, int* splitk) {
  const int order[] = {0, 1, 2, 4, 3};
  for (int oi = 0; oi < 5; ++oi) {
    const int c = order[oi];
    const long tiles = (long)((M + kShapes[c].bm - 1) / kShapes[c].bm) * ((N + kShapes[c].bn - 1) / kShapes[c].bn);
    if (tiles >= 240) {
      *cfg = c;
      *splitk = 1;
      return;
    }
  }
  // skinny: 64x64 tiles + split-K
  const long tiles = (long)((M + 63) / 64) * ((N + 63) / 64);
  int best = 1;
  for (int s : {2, 3, 4, 6, 8}) {
    if (K % (64 * s) != 0 || K / (64 * s) < 4) continue;
    best = s;
    if (tiles * s >= 240) break;
  }
  *cfg = (N % 8 == 0) ? 3 : 3;
  *splitk = (N % 8 == 0) ? best : 1;
}

size_t gemm_glds_workspace_bytes(int M, int N, int splitk) { return splitk > 1 ? (size_t)splitk * M * N * 4 : 0; }

bool launch_gemm_glds(const GemmArgs& a, int cfg, int splitk, void* workspace, hipStream_t s, const float* ln_colsum,
                      int ln_mode, float ln_eps, const int* rows) {
  float* ws = static_cast<float*>(workspace);
  const bool persist = cfg >= kGemmPersist && !rows;
  cfg &= kGemmPersist - 1;
  if (ln_mode != 0 && !a.ext_stats) {
    splitk = 1;  // in-kernel row statistics need the whole K range in one block
    if (kShapes[cfg < kNumCfg ? cfg : 3].bm * kShapes[cfg < kNumCfg ? cfg : 3].bn > 256 * 128) cfg = 0;
    if (cfg < kNumCfg && kKStep[cfg] != 64) cfg = 3;  // K groups: no in-kernel row statistics
  }
  // the SwiGLU epilogue pairs 16-column gate/up fragments: wave tiles must be multiples of 32
  // columns (configs 22-27, 38, 39: 48- / 144-column wave tiles; 36: 112)
  if (a.act == kActSwiglu && swiglu_bad(cfg)) cfg = kKStep[cfg] == 64 ? 3 : 17;
  return kLaunch[cfg < kNumCfg ? cfg : 3](a, splitk, ws, s, ln_colsum, ln_mode, ln_eps, rows, persist);
}

void launch_gemm_glds_grouped(const GemmArgs& a, int cfg, int n_groups, const int* offsets,
                              const unsigned long long* w_ptrs, const unsigned long long* c_ptrs, hipStream_t s,
                              const int* a_rows) {
  cfg &= kGemmPersist - 1;
  if (a.act == kActSwiglu && swiglu_bad(cfg)) cfg = kKStep[cfg] == 64 ? 3 : 17;
  kGrouped[cfg < kNumCfg ? cfg : 3](a, n_groups, offsets, w_ptrs, c_ptrs, s, a_rows);
}
