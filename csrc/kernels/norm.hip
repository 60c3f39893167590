// LayerNorm / RMSNorm, optionally fused with the residual add that precedes them.
//
// One row per WPR waves (WPR = 1 for H <= 2048, up to 4 for wide rows such as Llama's
// 4096): a 512-row activation then launches 512 x WPR waves instead of 512, so twice the
// SIMDs hold a wave and the row's loads are split WPR ways. Every global load of the row —
// x, the residual and the gain/bias vectors — is issued before the first reduction (one
// memory round trip, not two); the row stays in registers (16-B chunks, 8 bf16 per lane)
// between the statistics and the normalise pass, so it is read from HBM once. Statistics
// in fp32: wave xor-shuffle sums, then an LDS exchange across the row's waves. With a
// residual operand the kernel also writes the updated residual stream (x + r) — the
// executor's fused "add -> norm" node pairs.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int MAXC = 4;  // 16-B chunks per lane: H <= 8 * 64 * WPR * MAXC (8192 at WPR = 4)

template <bool RMS, int WPR>
__global__ __launch_bounds__(256) void norm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                   bf16* __restrict__ sum_out, const bf16* __restrict__ w,
                                                   const bf16* __restrict__ b, bf16* __restrict__ y, int M, int H,
                                                   float eps) {
  constexpr int RPB = 4 / WPR;  // rows per 256-thread block
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = wave % WPR;                 // this wave's slice of the row
  const int row = blockIdx.x * RPB + wave / WPR;
  const bool active = row < M;
  const int nch = H / 8;
  const int stride = 64 * WPR;
  const int base = sub * 64 + lane;
  const size_t roff = (size_t)(active ? row : 0) * H;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + roff);
  const bf16x8* rr = r ? reinterpret_cast<const bf16x8*>(r + roff) : nullptr;
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
  const bf16x8* br = b ? reinterpret_cast<const bf16x8*>(b) : nullptr;
  bf16x8 xa[MAXC], ra[MAXC], wa[MAXC], ba[MAXC];
  // issue every load first
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = base + c * stride;
    if (active && ch < nch) {
      xa[c] = xr[ch];
      if (rr) ra[c] = rr[ch];
      wa[c] = wr[ch];
      if (br) ba[c] = br[ch];
    }
  }
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = base + c * stride;
    if (active && ch < nch) {
      bf16x8 a = xa[c];
      if (rr) {
        bf16x8 sum;
#pragma unroll
        for (int e = 0; e < 8; ++e) sum[e] = f2bf(bf2f(a[e]) + bf2f(ra[c][e]));
        a = sum;
        if (sum_out) reinterpret_cast<bf16x8*>(sum_out + roff)[ch] = sum;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[c][e] = bf2f(a[e]);
        s += RMS ? v[c][e] * v[c][e] : v[c][e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] = 0.f;
    }
  }
  auto row_sum = [&](float t, int slot) {
    t = wave_sum(t);
    if (WPR == 1) return t;
    if (lane == 0) red[slot][wave] = t;
    __syncthreads();
    float tot = 0.f;
    const int w0 = (wave / WPR) * WPR;
#pragma unroll
    for (int k = 0; k < WPR; ++k) tot += red[slot][w0 + k];
    return tot;
  };
  s = row_sum(s, 0);
  float mean = 0.f, rstd;
  if (RMS) {
    rstd = rsqrtf(s / H + eps);
  } else {
    mean = s / H;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = base + c * stride;
      if (active && ch < nch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[c][e] - mean;
          q += d * d;
        }
      }
    }
    q = row_sum(q, 1);
    rstd = rsqrtf(q / H + eps);
  }
  if (!active) return;
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + roff);
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = base + c * stride;
    if (ch < nch) {
      bf16x8 out;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float o = (v[c][e] - mean) * rstd * bf2f(wa[c][e]);
        if (br) o += bf2f(ba[c][e]);
        out[e] = f2bf(o);
      }
      yr[ch] = out;
    }
  }
}

template <bool RMS>
void launch_norm(const void* x, const void* r, void* sum_out, const void* w, const void* b, void* y, int M, int H,
                 float eps, hipStream_t s) {
  // waves per row: enough that each lane holds <= MAXC chunks, and >= 2 for wide rows
  const int nch = H / 8;
  int wpr = 1;
  while (wpr < 4 && (nch > 64 * wpr * MAXC || (H >= 2048 && wpr * 1024 < H))) wpr *= 2;
  const dim3 block(256);
  const auto* xp = (const bf16*)x;
  const auto* rp = (const bf16*)r;
  auto* sp = (bf16*)sum_out;
  const auto* wp = (const bf16*)w;
  const auto* bp = (const bf16*)b;
  auto* yp = (bf16*)y;
  if (wpr == 1)
    hipLaunchKernelGGL((norm_kernel<RMS, 1>), dim3((M + 3) / 4), block, 0, s, xp, rp, sp, wp, bp, yp, M, H, eps);
  else if (wpr == 2)
    hipLaunchKernelGGL((norm_kernel<RMS, 2>), dim3((M + 1) / 2), block, 0, s, xp, rp, sp, wp, bp, yp, M, H, eps);
  else
    hipLaunchKernelGGL((norm_kernel<RMS, 4>), dim3(M), block, 0, s, xp, rp, sp, wp, bp, yp, M, H, eps);
}

}  // namespace

void launch_layernorm(const void* x, const void* r, void* sum_out, const void* w, const void* b, void* y, int M,
                      int H, float eps, hipStream_t s) {
  launch_norm<false>(x, r, sum_out, w, b, y, M, H, eps, s);
}

void launch_rmsnorm(const void* x, const void* r, void* sum_out, const void* w, void* y, int M, int H, float eps,
                    hipStream_t s) {
  launch_norm<true>(x, r, sum_out, w, nullptr, y, M, H, eps, s);
}
