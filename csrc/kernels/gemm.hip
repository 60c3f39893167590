// bf16 GEMM on MFMA with fused epilogues:  C = act(alpha * A @ W^T + bias) + R
//
//   A [M][K] row-major (activations), W [N][K] row-major (weights, K contiguous),
//   C, R [M][N], bias [N]; fp32 accumulation in the MFMA accumulators.
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop", 2-phase form of
// T3/T4): BK = 64 K-slices staged global -> registers -> LDS, double-buffered so the
// loads of slice k+1 are in flight while the MFMAs of slice k run, ONE barrier per
// slice. LDS rows are 128 B (64 bf16); 16-byte chunks are XOR-swizzled by (row & 7)
// so the 16 rows a ds_read_b128 lane group touches spread over the bank row
// (T2; <= 2-way instead of 8-way). Blocks are remapped XCD-aware (T1) so tiles that
// share a weight panel share an L2. The epilogue applies bias / GELU-tanh / SiLU /
// residual-add in registers before the single bf16 store, so "linear + activation"
// and "linear + residual" DAG nodes cost one kernel, not two or three.
//
// Tile configurations are chosen on the host per shape so that the grid covers the 256
// CUs: GPT-2's M = 512 projections are far too small for 128x128 tiles.
#include "common.h"
#include "kernels.h"

namespace {

template <int BM, int BN, int BK, int WAVES_M, int WAVES_N>
struct GemmCfg {
  static constexpr int T = 64 * WAVES_M * WAVES_N;
  static constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int CH = BK / 8;  // 16-byte chunks per LDS row
  static constexpr int A_PER = BM * CH / T, B_PER = BN * CH / T;
  static constexpr int STAGE = (BM + BN) * CH;  // bf16x8 units per buffer
  static_assert(FM >= 1 && FN >= 1, "wave tile too small");
  static_assert(A_PER >= 1 && B_PER >= 1 && A_PER * T == BM * CH && B_PER * T == BN * CH, "staging split");
  static_assert((CH & (CH - 1)) == 0, "BK/8 must be a power of two");
};

template <int BM, int BN, int BK, int WAVES_M, int WAVES_N>
__device__ __forceinline__ void gemm_tile(bf16x8* smem, const bf16* __restrict__ A, int lda,
                                          const bf16* __restrict__ W, int ldw, bf16* __restrict__ C, int ldc,
                                          const bf16* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M,
                                          int N, int K, int act, float alpha, int m0, int n0) {
  using G = GemmCfg<BM, BN, BK, WAVES_M, WAVES_N>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;

  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 ra[G::A_PER], rb[G::B_PER];
  const bf16x8 zero8 = {};

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < G::A_PER; ++i) {
      const int q = tid + i * G::T, row = q / G::CH, c = q % G::CH;
      const int gm = m0 + row, gk = k0 + c * 8;
      ra[i] = (gm < M && gk < K) ? *reinterpret_cast<const bf16x8*>(A + (size_t)gm * lda + gk) : zero8;
    }
#pragma unroll
    for (int i = 0; i < G::B_PER; ++i) {
      const int q = tid + i * G::T, row = q / G::CH, c = q % G::CH;
      const int gn = n0 + row, gk = k0 + c * 8;
      rb[i] = (gn < N && gk < K) ? *reinterpret_cast<const bf16x8*>(W + (size_t)gn * ldw + gk) : zero8;
    }
  };
  auto store_tile = [&](int buf) {
    bf16x8* s = smem + buf * G::STAGE;
#pragma unroll
    for (int i = 0; i < G::A_PER; ++i) {
      const int q = tid + i * G::T, row = q / G::CH, c = q % G::CH;
      s[row * G::CH + (c ^ (row & (G::CH - 1)))] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < G::B_PER; ++i) {
      const int q = tid + i * G::T, row = q / G::CH, c = q % G::CH;
      s[(BM + row) * G::CH + (c ^ (row & (G::CH - 1)))] = rb[i];
    }
  };

  const int nk = (K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile((kt + 1) * BK);  // in flight under the MFMAs below
    const bf16x8* s = smem + cur * G::STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 af[G::FM], bfg[G::FN];
#pragma unroll
      for (int i = 0; i < G::FM; ++i) {
        const int row = wm * G::WTM + i * 16 + (lane & 15);
        af[i] = s[row * G::CH + (chunk ^ (row & (G::CH - 1)))];
      }
#pragma unroll
      for (int j = 0; j < G::FN; ++j) {
        const int row = wn * G::WTN + j * 16 + (lane & 15);
        bfg[j] = s[(BM + row) * G::CH + (chunk ^ (row & (G::CH - 1)))];
      }
#pragma unroll
      for (int i = 0; i < G::FM; ++i)
#pragma unroll
        for (int j = 0; j < G::FN; ++j) acc[i][j] = mfma16x16x32(af[i], bfg[j], acc[i][j]);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // epilogue: alpha, bias, activation, residual, one bf16 store per element
#pragma unroll
  for (int j = 0; j < G::FN; ++j) {
    const int col = n0 + wn * G::WTN + j * 16 + (lane & 15);
    if (col >= N) continue;
    const float bv = bias ? bf2f(bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < G::FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * G::WTM + i * 16 + (lane >> 4) * 4 + r;
        if (row >= M) continue;
        float v = apply_act(alpha * acc[i][j][r] + bv, act);
        if (R) v += bf2f(R[(size_t)row * ldr + col]);
        C[(size_t)row * ldc + col] = f2bf(v);
      }
    }
  }
}

template <int BM, int BN, int BK, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_bf16_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ W, int ldw, bf16* __restrict__ C, int ldc,
    const bf16* __restrict__ bias, const bf16* __restrict__ R, int ldr, int M, int N, int K, int act, float alpha,
    int tiles_m, int tiles_n) {
  using G = GemmCfg<BM, BN, BK, WAVES_M, WAVES_N>;
  __shared__ bf16x8 smem[2 * G::STAGE];
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = bid % tiles_m, tn = bid / tiles_m;  // m fastest: XCD neighbours share the W panel
  gemm_tile<BM, BN, BK, WAVES_M, WAVES_N>(smem, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, act, alpha,
                                          tm * BM, tn * BN);
}

// Grouped (MoE expert) GEMM: rows of X are sorted by expert, offsets[E+1] delimit each
// expert's rows, W is [E][N][K]. grid.y = expert; blocks past an expert's row count exit.
template <int BM, int BN, int BK, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void grouped_gemm_kernel(
    const bf16* __restrict__ X, const int32_t* __restrict__ offsets, const bf16* __restrict__ W,
    bf16* __restrict__ Y, int N, int K, long ldw_expert, int act, int tiles_n) {
  using G = GemmCfg<BM, BN, BK, WAVES_M, WAVES_N>;
  __shared__ bf16x8 smem[2 * G::STAGE];
  const int e = blockIdx.y;
  const int r0 = offsets[e], r1 = offsets[e + 1];
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  if (tm * BM >= r1 - r0) return;
  gemm_tile<BM, BN, BK, WAVES_M, WAVES_N>(smem, X + (size_t)r0 * K, K, W + (size_t)e * ldw_expert, K,
                                          Y + (size_t)r0 * N, N, nullptr, nullptr, 0, r1 - r0, N, K, act, 1.0f,
                                          tm * BM, tn * BN);
}

template <int BM, int BN, int BK, int WM, int WN>
void launch_cfg(const GemmArgs& a, hipStream_t s) {
  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  dim3 grid(tiles_m * tiles_n), block(64 * WM * WN);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, BK, WM, WN>), grid, block, 0, s, (const bf16*)a.A, a.lda,
                     (const bf16*)a.W, a.ldw, (bf16*)a.C, a.ldc, (const bf16*)a.bias, (const bf16*)a.R, a.ldr, a.M,
                     a.N, a.K, a.act, a.alpha, tiles_m, tiles_n);
}

inline long blocks_for(int M, int N, int bm, int bn) { return (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn); }

}  // namespace

int gemm_pick_config(int M, int N, int K) {
  (void)K;
  // largest tile whose grid still covers the 256 CUs; smallest tile otherwise
  if (blocks_for(M, N, 128, 128) >= 256) return 0;
  if (blocks_for(M, N, 64, 128) >= 256) return 1;
  if (blocks_for(M, N, 64, 64) >= 256) return 2;
  return 3;
}

void launch_gemm_bf16(const GemmArgs& a, hipStream_t s) {
  const int cfg = a.config >= 0 ? a.config : gemm_pick_config(a.M, a.N, a.K);
  switch (cfg) {
    case 0: launch_cfg<128, 128, 64, 2, 2>(a, s); break;
    case 1: launch_cfg<64, 128, 64, 2, 2>(a, s); break;
    case 2: launch_cfg<64, 64, 64, 2, 2>(a, s); break;
    default: launch_cfg<32, 64, 64, 2, 2>(a, s); break;
  }
}

void launch_grouped_gemm(const void* X, const int32_t* offsets, const void* W, void* Y, int E, int N, int K,
                         int max_rows, int act, hipStream_t s) {
  // grid covers the worst case (all routed rows in one expert); idle tiles exit at once
  constexpr int BM = 64, BN = 64;
  const int tiles_m = (max_rows + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  dim3 grid(tiles_m * tiles_n, E), block(256);
  hipLaunchKernelGGL((grouped_gemm_kernel<BM, BN, 64, 2, 2>), grid, block, 0, s, (const bf16*)X, offsets,
                     (const bf16*)W, (bf16*)Y, N, K, (long)N * K, act, tiles_n);
}
