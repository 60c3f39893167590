// Mixture-of-experts routing kernels (Mixtral-style top-k):
//   router  : softmax over the E router logits, top-k, renormalised gate weights
//   align   : deterministic counting sort of the (token, k) assignments by expert ->
//             offsets[E+1], src_rows[slot] (token feeding each expert row), slot_of[m*k+j]
//   permute : gather token rows into expert-sorted order (16-B vectors per lane)
//   combine : y[m] = sum_j w[m][j] * expert_out[slot_of[m*k+j]]   (fp32 sum, bf16 out)
// Expert FFNs run as one grouped GEMM over the sorted rows (gemm.hip), so an EP edge
// in the DAG carries exactly the token subset routed to the experts placed on a GPU.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int MAX_E = 64;
constexpr int MAX_K = 8;

__global__ __launch_bounds__(256) void router_kernel(const bf16* __restrict__ logits, int M, int E, int topk,
                                                     int32_t* __restrict__ idx, float* __restrict__ w) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  float l[MAX_E];
  for (int e = 0; e < E; ++e) l[e] = bf2f(logits[(size_t)m * E + e]);
  int sel[MAX_K];
  float val[MAX_K];
  for (int j = 0; j < topk; ++j) {
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e) {
      bool taken = false;
      for (int q = 0; q < j; ++q) taken |= (sel[q] == e);
      if (!taken && (best < 0 || l[e] > bv)) {
        best = e;
        bv = l[e];
      }
    }
    sel[j] = best;
    val[j] = bv;
  }
  // softmax restricted to the selected experts (== full softmax renormalised over top-k)
  float mx = val[0], s = 0.f;
  for (int j = 0; j < topk; ++j) {
    val[j] = __expf(val[j] - mx);
    s += val[j];
  }
  for (int j = 0; j < topk; ++j) {
    idx[m * topk + j] = sel[j];
    w[m * topk + j] = val[j] / s;
  }
}

// single workgroup, 1024 threads: per expert a block-wide exclusive scan of "routed to e"
__global__ __launch_bounds__(1024) void align_kernel(const int32_t* __restrict__ idx, int n, int E,
                                                     int32_t* __restrict__ src_rows, int32_t* __restrict__ slot_of,
                                                     int32_t* __restrict__ offsets, int topk) {
  __shared__ int wave_tot[16];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int e = 0; e < E; ++e) {
    if (tid == 0) offsets[e] = base_s;
    for (int c0 = 0; c0 < n; c0 += 1024) {
      const int i = c0 + tid;
      const int f = (i < n && idx[i] == e) ? 1 : 0;
      // wave-level inclusive scan
      int x = f;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) wave_tot[wave] = x;
      __syncthreads();
      int pre = 0;
      for (int q = 0; q < wave; ++q) pre += wave_tot[q];
      const int base = base_s;
      if (f) {
        const int slot = base + pre + x - 1;
        src_rows[slot] = i / topk;
        slot_of[i] = slot;
      }
      __syncthreads();
      if (tid == 1023) base_s = base + pre + x;
      __syncthreads();
    }
  }
  if (tid == 0) offsets[E] = base_s;
}

__global__ __launch_bounds__(256) void permute_kernel(const bf16* __restrict__ x, const int32_t* __restrict__ src,
                                                      bf16* __restrict__ out, int rows, int H) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const bf16x8* in = reinterpret_cast<const bf16x8*>(x + (size_t)src[r] * H);
  bf16x8* o = reinterpret_cast<bf16x8*>(out + (size_t)r * H);
  for (int c = lane; c < H / 8; c += 64) o[c] = in[c];
}

// range (nullable, device int32[2]): only expert-sorted slots in [range[0], range[1]) count —
// one expert's share of the output (zero for tokens not routed to it)
__global__ __launch_bounds__(256) void combine_kernel(const bf16* __restrict__ eo, const int32_t* __restrict__ slot_of,
                                                      const float* __restrict__ w, bf16* __restrict__ y, int M,
                                                      int topk, int H, const int32_t* __restrict__ range) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const int r0 = range ? range[0] : 0, r1 = range ? range[1] : 0x7fffffff;
  bf16x8* yo = reinterpret_cast<bf16x8*>(y + (size_t)m * H);
  for (int c = lane; c < H / 8; c += 64) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < topk; ++j) {
      const int sl = slot_of[m * topk + j];
      if (sl < r0 || sl >= r1) continue;
      const float g = w[m * topk + j];
      const bf16x8 v = reinterpret_cast<const bf16x8*>(eo + (size_t)sl * H)[c];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += g * bf2f(v[e]);
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    yo[c] = o;
  }
}

// y[m] = r[m] + sum_j w[m,j] * E_{e}[slot[m,j] - off[e]],  e = idx[m,j]
// Expert outputs are COMPACT: expert e's node wrote its routed rows (expert-sorted order)
// to rows 0..count_e-1 of its own [M][H] buffer, wherever that buffer lives (a local arena
// view or an xGMI receive buffer). One wave per token row, 16-B chunks per lane.
__global__ __launch_bounds__(256) void gather_combine_kernel(const unsigned long long* __restrict__ eo_ptrs,
                                                             const int32_t* __restrict__ idx,
                                                             const int32_t* __restrict__ slot_of,
                                                             const int32_t* __restrict__ off,
                                                             const float* __restrict__ w, const bf16* __restrict__ r,
                                                             bf16* __restrict__ y, int M, int topk, int H, int E) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const bf16x8* src[8];
  float g[8];
  const int kk = topk < 8 ? topk : 8;
  for (int j = 0; j < kk; ++j) {
    const int e = idx[m * topk + j];
    const int row = slot_of[m * topk + j] - off[e];
    src[j] = (e >= 0 && e < E) ? reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(eo_ptrs[e]) +
                                                                   (size_t)row * H)
                               : nullptr;
    g[j] = w[m * topk + j];
  }
  bf16x8* yo = reinterpret_cast<bf16x8*>(y + (size_t)m * H);
  const bf16x8* ro = r ? reinterpret_cast<const bf16x8*>(r + (size_t)m * H) : nullptr;
  for (int c = lane; c < H / 8; c += 64) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ro) {
      const bf16x8 v = ro[c];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = bf2f(v[e]);
    }
    for (int j = 0; j < kk; ++j) {
      if (!src[j]) continue;
      const bf16x8 v = src[j][c];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += g[j] * bf2f(v[e]);
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    yo[c] = o;
  }
}

}  // namespace

void launch_moe_gather_combine(const unsigned long long* eo_ptrs, const int32_t* idx, const int32_t* slot_of,
                               const int32_t* off, const float* w, const void* r, void* y, int M, int topk, int H,
                               int E, hipStream_t s) {
  hipLaunchKernelGGL(gather_combine_kernel, dim3((M + 3) / 4), dim3(256), 0, s, eo_ptrs, idx, slot_of, off, w,
                     (const bf16*)r, (bf16*)y, M, topk, H, E);
}

void launch_moe_router(const void* logits, int M, int E, int topk, int32_t* topk_idx, float* topk_w,
                       hipStream_t s) {
  hipLaunchKernelGGL(router_kernel, dim3((M + 255) / 256), dim3(256), 0, s, (const bf16*)logits, M, E, topk, topk_idx,
                     topk_w);
}

void launch_moe_align(const int32_t* topk_idx, int M, int topk, int E, int32_t* src_rows, int32_t* slot_of,
                      int32_t* offsets, hipStream_t s) {
  hipLaunchKernelGGL(align_kernel, dim3(1), dim3(1024), 0, s, topk_idx, M * topk, E, src_rows, slot_of, offsets,
                     topk);
}

void launch_moe_permute(const void* x, const int32_t* src_rows, void* out, int rows, int H, hipStream_t s) {
  hipLaunchKernelGGL(permute_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, (const bf16*)x, src_rows, (bf16*)out,
                     rows, H);
}

void launch_moe_combine(const void* expert_out, const int32_t* slot_of, const float* weights, void* y, int M,
                        int topk, int H, const int32_t* range, hipStream_t s) {
  hipLaunchKernelGGL(combine_kernel, dim3((M + 3) / 4), dim3(256), 0, s, (const bf16*)expert_out, slot_of, weights,
                     (bf16*)y, M, topk, H, range);
}
