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

// Router + align fused into ONE workgroup: per token the top-k experts (router_kernel's
// selection: ties go to the lower expert index) and renormalised gates, then the counting sort
// of the M*k assignments by expert in align_kernel's order (stable in assignment index i =
// m*k + j), so the outputs equal the two-launch pair exactly. The experts of the assignments
// stay in LDS; ranks within a 64-assignment wave come from one ballot per expert, wave
// prefixes from an LDS table: two barriers per 1024 assignments instead of three per expert.
__global__ __launch_bounds__(1024) void route_kernel(const bf16* __restrict__ logits, int M, int E, int topk,
                                                     int32_t* __restrict__ idx, float* __restrict__ w,
                                                     int32_t* __restrict__ src_rows, int32_t* __restrict__ slot_of,
                                                     int32_t* __restrict__ offsets) {
  __shared__ unsigned char es[kRouteMaxAssign];  // expert of each assignment (E <= 64)
  __shared__ int base[MAX_E];                    // per expert: first slot of the current chunk
  __shared__ int wcnt[16][MAX_E];                // per wave, per expert: assignments in the chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = M * topk;
  if (tid < MAX_E) base[tid] = 0;
  __syncthreads();
  for (int m = tid; m < M; m += 1024) {
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
    float mx = val[0], sum = 0.f;
    for (int j = 0; j < topk; ++j) {
      val[j] = __expf(val[j] - mx);
      sum += val[j];
    }
    for (int j = 0; j < topk; ++j) {
      idx[m * topk + j] = sel[j];
      w[m * topk + j] = val[j] / sum;
      es[m * topk + j] = (unsigned char)sel[j];
      atomicAdd(&base[sel[j]], 1);  // per-expert totals (order-free)
    }
  }
  __syncthreads();
  if (wave == 0) {  // exclusive scan of the E <= 64 totals -> offsets, first slots
    const int c = lane < E ? base[lane] : 0;
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane < E) {
      offsets[lane] = x - c;
      base[lane] = x - c;
    }
    if (lane == 63) offsets[E] = x;
  }
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int i = c0 + tid;
    const int e = i < n ? (int)es[i] : -1;
    int rank = 0;
    for (int q = 0; q < E; ++q) {
      const unsigned long long b = __ballot(e == q);
      if (lane == 0) wcnt[wave][q] = __popcll(b);
      if (e == q) rank = __popcll(b & ((1ull << lane) - 1ull));
    }
    __syncthreads();
    if (e >= 0) {
      int slot = base[e] + rank;
      for (int v = 0; v < wave; ++v) slot += wcnt[v][e];
      src_rows[slot] = i / topk;
      slot_of[i] = slot;
    }
    __syncthreads();
    if (tid < E) {
      int t = 0;
      for (int v = 0; v < 16; ++v) t += wcnt[v][tid];
      base[tid] += t;
    }
    __syncthreads();
  }
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
// view or an xGMI receive buffer). One workgroup per token row: the routing words are
// block-uniform (scalar loads), and each thread issues all k + 1 of its 16-B loads before the
// arithmetic, so a 4096-wide row is 2 load batches per thread (a wave per row took 8 dependent
// rounds: 15 us per Mixtral layer at 1 TB/s).
__global__ __launch_bounds__(256) void gather_combine_kernel(const unsigned long long* __restrict__ eo_ptrs,
                                                             const int32_t* __restrict__ idx,
                                                             const int32_t* __restrict__ slot_of,
                                                             const int32_t* __restrict__ off,
                                                             const float* __restrict__ w, const bf16* __restrict__ r,
                                                             bf16* __restrict__ y, int M, int topk, int H, int E) {
  const int m = blockIdx.x;
  const bf16x8* src[MAX_K];
  float g[MAX_K];
  const int kk = topk < MAX_K ? topk : MAX_K;
#pragma unroll
  for (int j = 0; j < MAX_K; ++j) {
    src[j] = nullptr;
    g[j] = 0.f;
    if (j >= kk) continue;
    const int e = idx[m * topk + j];
    if (e < 0 || e >= E) continue;
    const int row = slot_of[m * topk + j] - off[e];
    src[j] = reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(eo_ptrs[e]) + (size_t)row * H);
    g[j] = w[m * topk + j];
  }
  bf16x8* yo = reinterpret_cast<bf16x8*>(y + (size_t)m * H);
  const bf16x8* ro = r ? reinterpret_cast<const bf16x8*>(r + (size_t)m * H) : nullptr;
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    bf16x8 v[MAX_K];
    bf16x8 rv = {};
#pragma unroll
    for (int j = 0; j < MAX_K; ++j)
      if (src[j]) v[j] = src[j][c];
    if (ro) rv = ro[c];
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = ro ? bf2f(rv[e]) : 0.f;
#pragma unroll
    for (int j = 0; j < MAX_K; ++j) {
      if (!src[j]) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += g[j] * bf2f(v[j][e]);
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
  hipLaunchKernelGGL(gather_combine_kernel, dim3(M), dim3(256), 0, s, eo_ptrs, idx, slot_of, off, w,
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

void launch_moe_route(const void* logits, int M, int E, int topk, int32_t* topk_idx, float* topk_w,
                      int32_t* src_rows, int32_t* slot_of, int32_t* offsets, hipStream_t s) {
  hipLaunchKernelGGL(route_kernel, dim3(1), dim3(1024), 0, s, (const bf16*)logits, M, E, topk, topk_idx, topk_w,
                     src_rows, slot_of, offsets);
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
