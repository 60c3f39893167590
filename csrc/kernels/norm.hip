// LayerNorm / RMSNorm, optionally fused with the residual add that precedes them.
//
// One wave per row, 4 rows per 256-thread block; each lane owns 16-byte chunks
// (8 bf16) of the row, kept in registers between the statistics pass and the
// normalise pass so the row is read from HBM exactly once. fp32 statistics via
// wave-wide xor shuffles (64 lanes). With a residual operand the kernel writes both the
// updated residual stream (x + r) and its normalised form, which is how the executor
// fuses the GPT-2 "attn_residual -> ln2" / Llama "add -> rmsnorm" DAG node pairs into
// one pass.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int MAXC = 16;  // up to 16 chunks/lane -> H <= 8192

template <bool RMS>
__global__ __launch_bounds__(256) void norm_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                   bf16* __restrict__ sum_out, const bf16* __restrict__ w,
                                                   const bf16* __restrict__ b, bf16* __restrict__ y, int M, int H,
                                                   float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = H / 8;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)row * H);
  const bf16x8* rr = r ? reinterpret_cast<const bf16x8*>(r + (size_t)row * H) : nullptr;
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      bf16x8 a = xr[ch];
      if (rr) {
        const bf16x8 bb = rr[ch];
        bf16x8 sum;
#pragma unroll
        for (int e = 0; e < 8; ++e) sum[e] = f2bf(bf2f(a[e]) + bf2f(bb[e]));
        a = sum;
        if (sum_out) reinterpret_cast<bf16x8*>(sum_out + (size_t)row * H)[ch] = sum;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[c][e] = bf2f(a[e]);
        s += RMS ? v[c][e] * v[c][e] : v[c][e];
      }
    }
  }
  s = wave_sum(s);
  float mean = 0.f, rstd;
  if (RMS) {
    rstd = rsqrtf(s / H + eps);
  } else {
    mean = s / H;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[c][e] - mean;
          q += d * d;
        }
      }
    }
    q = wave_sum(q);
    rstd = rsqrtf(q / H + eps);
  }
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
  const bf16x8* br = b ? reinterpret_cast<const bf16x8*>(b) : nullptr;
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + (size_t)row * H);
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      const bf16x8 wv = wr[ch];
      bf16x8 out;
      if (br) {
        const bf16x8 bv = br[ch];
#pragma unroll
        for (int e = 0; e < 8; ++e) out[e] = f2bf((v[c][e] - mean) * rstd * bf2f(wv[e]) + bf2f(bv[e]));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) out[e] = f2bf((v[c][e] - mean) * rstd * bf2f(wv[e]));
      }
      yr[ch] = out;
    }
  }
}

}  // namespace

void launch_layernorm(const void* x, const void* r, void* sum_out, const void* w, const void* b, void* y, int M,
                      int H, float eps, hipStream_t s) {
  hipLaunchKernelGGL(norm_kernel<false>, dim3((M + 3) / 4), dim3(256), 0, s, (const bf16*)x, (const bf16*)r,
                     (bf16*)sum_out, (const bf16*)w, (const bf16*)b, (bf16*)y, M, H, eps);
}

void launch_rmsnorm(const void* x, const void* r, void* sum_out, const void* w, void* y, int M, int H, float eps,
                    hipStream_t s) {
  hipLaunchKernelGGL(norm_kernel<true>, dim3((M + 3) / 4), dim3(256), 0, s, (const bf16*)x, (const bf16*)r,
                     (bf16*)sum_out, (const bf16*)w, (const bf16*)nullptr, (bf16*)y, M, H, eps);
}
