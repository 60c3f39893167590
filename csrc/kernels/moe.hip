// Mixture-of-experts routing kernels (Mixtral-style top-k):
//   router  : softmax over the E router logits, top-k, renormalised gate weights
//   align   : deterministic counting sort of the (token, k) assignments by expert ->
//             offsets[E+1], src_rows[slot] (token feeding each expert row), slot_of[m*k+j]
//   permute : gather token rows into expert-sorted order (16-B vectors per lane)
//   combine : y[m] = sum_j w[m][j] * expert_out[slot_of[m*k+j]]   (fp32 sum, bf16 out)
// Expert FFNs run as one grouped GEMM over the sorted rows (gemm.hip), so an EP edge
// in the DAG carries exactly the token subset routed to the experts placed on a GPU.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace {

constexpr int MAX_E = 64;
constexpr int MAX_K = 8;

// top-k of one token's E logits: ties go to the lower expert index; gates = softmax over the
// selected logits (== the full softmax renormalised over the top-k). The j loop is unrolled to
// MAX_K so sel / val stay in registers, and taken experts are a bitmask: a runtime-indexed
// float[E] / int[k] lived in scratch memory (272 B per lane).
__device__ __forceinline__ void select_topk(const bf16* __restrict__ lrow, int E, int topk, int (&sel)[MAX_K],
                                            float (&val)[MAX_K]) {
  unsigned long long taken = 0ull;
#pragma unroll
  for (int j = 0; j < MAX_K; ++j) {
    sel[j] = 0;
    val[j] = 0.f;
    if (j >= topk) continue;
    int best = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e) {
      const float le = bf2f(lrow[e]);
      if (!((taken >> e) & 1ull) && (best < 0 || le > bv)) {
        best = e;
        bv = le;
      }
    }
    taken |= 1ull << best;
    sel[j] = best;
    val[j] = bv;
  }
  const float mx = val[0];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAX_K; ++j)
    if (j < topk) {
      val[j] = __expf(val[j] - mx);
      s += val[j];
    }
#pragma unroll
  for (int j = 0; j < MAX_K; ++j)
    if (j < topk) val[j] /= s;
}

__global__ __launch_bounds__(256) void router_kernel(const bf16* __restrict__ logits, int M, int E, int topk,
                                                     int32_t* __restrict__ idx, float* __restrict__ w) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  int sel[MAX_K];
  float val[MAX_K];
  select_topk(logits + (size_t)m * E, E, topk, sel, val);
#pragma unroll
  for (int j = 0; j < MAX_K; ++j)
    if (j < topk) {
      idx[m * topk + j] = sel[j];
      w[m * topk + j] = val[j];
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

// Router + align for one MoE layer inside ONE workgroup of NT threads: per token the top-k
// experts and renormalised gates (select_topk), then the counting sort of the M*k assignments
// by expert in align_kernel's order (stable in assignment index i = m*k + j), so the outputs
// equal the router_kernel + align_kernel pair exactly. The experts of the assignments stay in
// LDS; ranks within a 64-assignment wave come from one ballot per expert, wave prefixes from an
// LDS table: two barriers per NT assignments instead of three per expert.
template <int NT>
__device__ __forceinline__ void route_block(const bf16* __restrict__ logits, int M, int E, int topk,
                                            int32_t* __restrict__ idx, float* __restrict__ w,
                                            int32_t* __restrict__ src_rows, int32_t* __restrict__ slot_of,
                                            int32_t* __restrict__ offsets, unsigned char* es, int* base,
                                            int (*wcnt)[MAX_E]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = M * topk;
  if (tid < MAX_E) base[tid] = 0;
  __syncthreads();
  for (int m = tid; m < M; m += NT) {
    int sel[MAX_K];
    float val[MAX_K];
    select_topk(logits + (size_t)m * E, E, topk, sel, val);
#pragma unroll
    for (int j = 0; j < MAX_K; ++j)
      if (j < topk) {
        idx[m * topk + j] = sel[j];
        w[m * topk + j] = val[j];
        es[m * topk + j] = (unsigned char)sel[j];
      }
  }
  __syncthreads();
  // per-expert totals: one ballot per expert per wave, one LDS add per (wave, expert) — an
  // LDS atomic per assignment piles 128 same-address atomics on each expert's counter
  for (int c0 = 0; c0 < n; c0 += NT) {
    const int i = c0 + tid;
    const int e = i < n ? (int)es[i] : -1;
    for (int q = 0; q < E; ++q) {
      const unsigned long long b = __ballot(e == q);
      if (lane == 0 && b) atomicAdd(&base[q], __popcll(b));
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
  for (int c0 = 0; c0 < n; c0 += NT) {
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
      for (int v = 0; v < NT / 64; ++v) t += wcnt[v][tid];
      base[tid] += t;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void route_kernel(const bf16* __restrict__ logits, int M, int E, int topk,
                                                     int32_t* __restrict__ idx, float* __restrict__ w,
                                                     int32_t* __restrict__ src_rows, int32_t* __restrict__ slot_of,
                                                     int32_t* __restrict__ offsets) {
  __shared__ unsigned char es[kRouteMaxAssign];  // expert of each assignment (E <= 64)
  __shared__ int base[MAX_E];                    // per expert: first slot of the current chunk
  __shared__ int wcnt[16][MAX_E];                // per wave, per expert: assignments in the chunk
  route_block<1024>(logits, M, E, topk, idx, w, src_rows, slot_of, offsets, es, base, wcnt);
}

// Router GEMM + routing in ONE launch (replaces a split-K GEMM, its reduce and the route
// kernel: 6.2 + 5.8 + 8.3 us per Mixtral layer). A workgroup of 8 waves takes GR_TOK tokens;
// wave v computes the logits of token v / GR_EW for experts (v % GR_EW) * EPW .. + EPW - 1
// straight from global memory (fp32 dot products over 16-B chunks, one wave reduction per
// expert): M / GR_TOK workgroups cover the chip, each wave loads its x row and its weight
// rows in one round trip. The logits are published with agent-scope (write-through) stores
// and every workgroup draws a ticket; the LAST one routes every token from the published
// logits (route_block) and resets the ticket. No workgroup waits on another, and nothing is
// fenced (a device-scope fence writes back this XCD's whole L2: 36 us for the launch).
constexpr int GR_WAVES = 8;
constexpr int GR_XV = 8;  // 16-B x chunks per lane (H <= 8 * 64 * 8 = 4096)
template <int EPW, int GR_EW>  // experts per wave, waves per token (EPW * GR_EW >= E)
__global__ __launch_bounds__(64 * GR_WAVES) void gate_route_kernel(
    const bf16* __restrict__ x, int ldx, const bf16* __restrict__ wg, int M, int H, int E, int topk,
    bf16* __restrict__ logits, int* __restrict__ ticket, int32_t* __restrict__ idx, float* __restrict__ w,
    int32_t* __restrict__ src_rows, int32_t* __restrict__ slot_of, int32_t* __restrict__ offsets) {
  constexpr int NT = 64 * GR_WAVES, GR_TOK = GR_WAVES / GR_EW;
  __shared__ unsigned char es[kRouteMaxAssign];
  __shared__ unsigned int lg[kRouteMaxAssign / 2];  // the last block's copy of all logits (bf16 pairs)
  __shared__ int base[MAX_E];
  __shared__ int wcnt[GR_WAVES][MAX_E];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hv = H / 8;
  const int m = blockIdx.x * GR_TOK + wave / GR_EW, e0 = (wave % GR_EW) * EPW;
  if (m < M && e0 < E) {  // wave-uniform
    // one round trip: the token row and this wave's weight rows (clamped, not guarded: a
    // branch per load serialises them)
    const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)m * ldx);
    bf16x8 xv[GR_XV], wv[EPW][GR_XV];
#pragma unroll
    for (int u = 0; u < GR_XV; ++u) xv[u] = xr[min(u * 64 + lane, hv - 1)];
#pragma unroll
    for (int k = 0; k < EPW; ++k) {
      const bf16x8* wr = reinterpret_cast<const bf16x8*>(wg + (size_t)min(e0 + k, E - 1) * H);
#pragma unroll
      for (int u = 0; u < GR_XV; ++u) wv[k][u] = wr[min(u * 64 + lane, hv - 1)];
    }
    float acc[EPW];
#pragma unroll
    for (int k = 0; k < EPW; ++k) acc[k] = 0.f;
    __builtin_amdgcn_sched_barrier(0);  // every load above is issued before the first use
#pragma unroll
    for (int u = 0; u < GR_XV; ++u) {
      const bool in = u * 64 + lane < hv;  // a select, not a branch (a break sinks the loads)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float xf = in ? bf2f(xv[u][q]) : 0.f;
#pragma unroll
        for (int k = 0; k < EPW; ++k) acc[k] += xf * bf2f(wv[k][u][q]);
      }
    }
#pragma unroll
    for (int k = 0; k < EPW; k += 2) {
      if (e0 + k >= E) break;
      const float t0 = wave_sum(acc[k]), t1 = wave_sum(acc[k + 1]);
      if (lane == 0) {
        const unsigned int pr = (unsigned int)__builtin_bit_cast(unsigned short, f2bf(t0)) |
                                ((unsigned int)__builtin_bit_cast(unsigned short, f2bf(t1)) << 16);
        __hip_atomic_store(reinterpret_cast<unsigned int*>(logits) + ((size_t)m * E + e0 + k) / 2, pr,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // Hand-off (MI355X_MICROARCH.md, "Valid forms", first row of the sc1 table — measured on
  // gfx950 / ROCm 7.2, not an architectural guarantee): every logit is stored write-through
  // (agent-scope relaxed 4-B store = global_store sc1), each storing wave drains its stores,
  // ONE lane per workgroup adds to the unsharded ticket after the workgroup barrier, and only
  // the workgroup whose add returns gridDim-1 reads the logits — with sc1 loads (agent-scope
  // relaxed), so no L1 line can be stale. A release/acquire fence pair would write back and
  // invalidate this XCD's caches per workgroup (36 us per launch measured with
  // __threadfence); tests/test_kernels_gpu.py::test_moe_gate_route_many_blocks checks the
  // hand-off at the largest M (1024 workgroups) with fresh logits every launch, under uneven load.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's logits stores are complete
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (int)gridDim.x - 1;
    if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  }
  __syncthreads();
  if (!last) return;  // block-uniform
  // agent-scope loads: the other blocks' logits come from memory, never from a stale cache line
  const int nl = M * E / 2;
  for (int i0 = 0; i0 < nl; i0 += NT * 8) {
    unsigned int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = __hip_atomic_load(reinterpret_cast<const unsigned int*>(logits) + min(i0 + u * NT + tid, nl - 1),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u * NT + tid < nl) lg[i0 + u * NT + tid] = v[u];
  }
  __syncthreads();
  route_block<NT>(reinterpret_cast<const bf16*>(lg), M, E, topk, idx, w, src_rows, slot_of, offsets, es, base,
                  wcnt);
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
constexpr int GC_MAXV = 4;  // 8-column vectors per thread: H <= 256 * 8 * GC_MAXV
// KK expert slots (>= top-k; unused slots and unrouted experts read a valid row with weight 0)
// and VPT vectors per thread at compile time: every load of the row is issued before the
// first use, with no branch around any of them (a null-checked load per expert made the
// compiler wait a full memory latency per load)
template <int KK, int VPT>
__global__ __launch_bounds__(256) void gather_combine_kernel(const unsigned long long* __restrict__ eo_ptrs,
                                                             const int32_t* __restrict__ idx,
                                                             const int32_t* __restrict__ slot_of,
                                                             const int32_t* __restrict__ off,
                                                             const float* __restrict__ w, const bf16* __restrict__ r,
                                                             bf16* __restrict__ y, int M, int topk, int H, int E,
                                                             bf16* __restrict__ yn, const bf16* __restrict__ nw,
                                                             const bf16* __restrict__ nb, int nmode, float neps) {
  __shared__ float red[2][4];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16* rrow = r ? r + (size_t)m * H : nullptr;
  const bf16* src[KK];
  float g[KK];
  bool ok[KK];  // slot j holds a routed expert row (padding slots j >= topk and invalid experts do not)
  const bf16* any_row = nullptr;
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    src[j] = nullptr;
    g[j] = 0.f;
    ok[j] = false;
    if (j >= topk) continue;
    const int e = idx[m * topk + j];
    if (e < 0 || e >= E) continue;
    src[j] = reinterpret_cast<const bf16*>(eo_ptrs[e]) + (size_t)(slot_of[m * topk + j] - off[e]) * H;
    g[j] = w[m * topk + j];
    ok[j] = true;
    any_row = src[j];
  }
  // a row every unused load may read: a routed row, the residual, or row 0 of expert 0's buffer
  // (allocated memory) — never the uninitialised output row; what such a load returns is
  // discarded by a select below (0 * NaN would not be)
  if (!any_row) any_row = rrow ? rrow : reinterpret_cast<const bf16*>(eo_ptrs[0]);
#pragma unroll
  for (int j = 0; j < KK; ++j)
    if (!src[j]) src[j] = any_row;
  const bf16* rsrc = rrow ? rrow : any_row;
  const bool has_r = rrow != nullptr;
  const int nv = H / 8;
  bf16x8 v[VPT][KK], rv[VPT];
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const int cl = min(u * 256 + tid, nv - 1);  // clamped loads, guarded stores
#pragma unroll
    for (int j = 0; j < KK; ++j) v[u][j] = reinterpret_cast<const bf16x8*>(src[j])[cl];
    rv[u] = reinterpret_cast<const bf16x8*>(rsrc)[cl];
  }
  bf16x8* yo = reinterpret_cast<bf16x8*>(y + (size_t)m * H);
  float yv[VPT][8];
  float s1 = 0.f;
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const int c = u * 256 + tid;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = has_r ? bf2f(rv[u][e]) : 0.f;
#pragma unroll
    for (int j = 0; j < KK; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += ok[j] ? g[j] * bf2f(v[u][j][e]) : 0.f;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf(acc[e]);
      yv[u][e] = c < nv ? bf2f(o[e]) : 0.f;
      s1 += yv[u][e];
    }
    if (c < nv) yo[c] = o;
  }
  if (!yn) return;  // block-uniform
  // post-norm for the next (unfolded) norm: this workgroup owns the whole row; its weights are
  // requested before the two reductions
  bf16x8 wv[VPT], bv[VPT];
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const int cl = min(u * 256 + tid, nv - 1);
    wv[u] = reinterpret_cast<const bf16x8*>(nw)[cl];
    bv[u] = nb ? reinterpret_cast<const bf16x8*>(nb)[cl] : bf16x8{};
  }
  auto block_sum = [&](float t, int slot) {
    t = wave_sum(t);
    if (lane == 0) red[slot][wave] = t;
    __syncthreads();
    return red[slot][0] + red[slot][1] + red[slot][2] + red[slot][3];
  };
  const float inv_h = 1.0f / (float)H;
  float mean = 0.f;
  if (nmode == 1) mean = block_sum(s1, 0) * inv_h;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < VPT; ++u)
    if (u * 256 + tid < nv)
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (yv[u][e] - mean) * (yv[u][e] - mean);
  const float rstd = rsqrtf(block_sum(q, 1) * inv_h + neps);
  bf16x8* yno = reinterpret_cast<bf16x8*>(yn + (size_t)m * H);
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    const int c = u * 256 + tid;
    if (c >= nv) continue;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = (yv[u][e] - mean) * rstd * bf2f(wv[u][e]);
      if (nb) t += bf2f(bv[u][e]);
      o[e] = f2bf(t);
    }
    yno[c] = o;
  }
}

}  // namespace

void launch_moe_gather_combine(const unsigned long long* eo_ptrs, const int32_t* idx, const int32_t* slot_of,
                               const int32_t* off, const float* w, const void* r, void* y, int M, int topk, int H,
                               int E, hipStream_t s, void* yn, const void* nw, const void* nb, int nmode,
                               float neps) {
#define DLS_GC(KK, VPT)                                                                                            \
  hipLaunchKernelGGL((gather_combine_kernel<KK, VPT>), dim3(M), dim3(256), 0, s, eo_ptrs, idx, slot_of, off, w,      \
                     (const bf16*)r, (bf16*)y, M, topk, H, E, (bf16*)yn, (const bf16*)nw, (const bf16*)nb, nmode, \
                     neps)
#define DLS_GC_K(VPT)          \
  if (topk <= 1) DLS_GC(1, VPT); \
  else if (topk <= 2) DLS_GC(2, VPT); \
  else if (topk <= 4) DLS_GC(4, VPT); \
  else DLS_GC(8, VPT)
  if (H <= 256 * 8 * 2) {
    DLS_GC_K(2);
  } else {
    DLS_GC_K(4);
  }
#undef DLS_GC_K
#undef DLS_GC
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

bool launch_moe_gate_route(const void* x, int ldx, const void* wg, int M, int H, int E, int topk, void* logits,
                           int* ticket, int32_t* topk_idx, float* topk_w, int32_t* src_rows, int32_t* slot_of,
                           int32_t* offsets, hipStream_t s) {
  if (H > 64 * 8 * GR_XV || M * topk > kRouteMaxAssign || M * E > kRouteMaxAssign || E % 2 || H % 8 || E > 16 ||
      ldx % 8 || reinterpret_cast<uintptr_t>(x) % 16 || reinterpret_cast<uintptr_t>(wg) % 16 ||
      reinterpret_cast<uintptr_t>(logits) % 4)
    return false;  // 16-B vector loads, 4-B logits pair stores
  // 2 experts per wave: E = 8 -> 4 waves per token, 2 tokens per workgroup (256 workgroups
  // for a 512-token batch); E <= 16 -> 8 waves per token
#define DLS_GR(EPW, EW)                                                                                           \
  hipLaunchKernelGGL((gate_route_kernel<EPW, EW>), dim3((M + GR_WAVES / EW - 1) / (GR_WAVES / EW)),               \
                     dim3(64 * GR_WAVES), 0, s, (const bf16*)x, ldx, (const bf16*)wg, M, H, E, topk, (bf16*)logits, \
                     ticket, topk_idx, topk_w, src_rows, slot_of, offsets)
  if (E <= 8) DLS_GR(2, 4);
  else DLS_GR(2, 8);
#undef DLS_GR
  return true;
}

void launch_moe_permute(const void* x, const int32_t* src_rows, void* out, int rows, int H, hipStream_t s) {
  hipLaunchKernelGGL(permute_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, (const bf16*)x, src_rows, (bf16*)out,
                     rows, H);
}

// Cross-request expert batch (executor._run_moe_xbatch): group g is one (request, expert) pair
// placed on this GPU; its rows are rows [off_q[e], off_q[e+1]) of request q's expert-sorted block,
// which starts at row base[q] of the batch's token matrix. One workgroup writes the groups'
// offsets (prefix sums of their device-side counts) and every sorted row's token row, so ONE
// grouped launch pair runs all of them with each weight panel streamed once (no host sync).
__global__ __launch_bounds__(256) void xbatch_index_kernel(XbatchIndexArgs a) {
  __shared__ int lo[kXbatchMaxGroups];
  __shared__ int start[kXbatchMaxGroups + 1];
  const int t = threadIdx.x;
  if (t < a.G) {
    const int32_t* off = a.off[a.req[t]];
    const int e = a.expert[t];
    lo[t] = a.base[a.req[t]] + off[e];
    start[t + 1] = off[e + 1] - off[e];
  }
  __syncthreads();
  if (t == 0) {
    start[0] = 0;
    for (int g = 0; g < a.G; ++g) start[g + 1] += start[g];
  }
  __syncthreads();
  if (t <= a.G) a.offsets[t] = start[t];
  for (int g = 0; g < a.G; ++g) {
    const int n = start[g + 1] - start[g];
    for (int r = t; r < n; r += 256) a.a_rows[start[g] + r] = lo[g] + r;
  }
}

// Capacity edges (see kernels.h MoePackArgs): block (x, d) moves rows x, x + gridDim.x, ... of
// destination d, one wave per row, 16-B vectors per lane. Every block recomputes d's segment
// table from the device offsets (n_exp <= 8 experts: a few scalar loads).
__global__ __launch_bounds__(256) void moe_pack_kernel(bf16* __restrict__ x, int H, const int32_t* __restrict__ src,
                                                       const int32_t* __restrict__ off, MoePackArgs a,
                                                       int32_t* __restrict__ ovf, int unpack) {
  const MoePackDest& d = a.d[blockIdx.y];
  int lo[kMoePackMaxExp], cum[kMoePackMaxExp + 1];
  cum[0] = 0;
#pragma unroll
  for (int k = 0; k < kMoePackMaxExp; ++k) {
    const int e = k < d.n_exp ? d.experts[k] : 0;
    const int n = k < d.n_exp ? off[e + 1] - off[e] : 0;
    lo[k] = k < d.n_exp ? off[e] : 0;
    cum[k + 1] = cum[k] + n;
    if (blockIdx.x == 0 && threadIdx.x == 0 && k < d.n_exp && d.eflag[k] >= 0 && n > d.ecap[k]) ovf[d.eflag[k]] = 1;
  }
  const int total = cum[kMoePackMaxExp];
  if (blockIdx.x == 0 && threadIdx.x == 0 && total > d.cap && d.flag >= 0) ovf[d.flag] = 1;
  const int rows = min(total, d.cap);
  const int lane = threadIdx.x & 63;
  bf16* buf = static_cast<bf16*>(d.buf);
  for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < rows; c += gridDim.x * 4) {
    int k = 0;
#pragma unroll
    for (int q = 1; q < kMoePackMaxExp; ++q) k += (c >= cum[q]) ? 1 : 0;
    const int j = lo[k] + c - cum[k];  // position in the expert-sorted order
    bf16x8* cp = reinterpret_cast<bf16x8*>(buf + (size_t)c * H);
    if (unpack) {
      bf16x8* xp = reinterpret_cast<bf16x8*>(x + (size_t)j * H);
      for (int v = lane; v < H / 8; v += 64) xp[v] = cp[v];
    } else {
      const bf16x8* xp = reinterpret_cast<const bf16x8*>(x + (size_t)src[j] * H);
      for (int v = lane; v < H / 8; v += 64) cp[v] = xp[v];
    }
  }
}

void launch_moe_xbatch_index(const XbatchIndexArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(xbatch_index_kernel, dim3(1), dim3(256), 0, s, a);
}

void launch_moe_combine(const void* expert_out, const int32_t* slot_of, const float* weights, void* y, int M,
                        int topk, int H, const int32_t* range, hipStream_t s) {
  hipLaunchKernelGGL(combine_kernel, dim3((M + 3) / 4), dim3(256), 0, s, (const bf16*)expert_out, slot_of, weights,
                     (bf16*)y, M, topk, H, range);
}

void launch_moe_pack(const void* x, int H, const int32_t* src_rows, const int32_t* offsets, const MoePackArgs& a,
                     int32_t* ovf, int unpack, int max_rows, hipStream_t s) {
  // blocks per destination: enough waves for the largest capacity (4 rows per block)
  const int bx = std::max(1, std::min(64, (max_rows + 3) / 4));
  hipLaunchKernelGGL(moe_pack_kernel, dim3(bx, a.n), dim3(256), 0, s, (bf16*)x, H, src_rows, offsets, a, ovf, unpack);
}
