// A pre-norm attention block as ONE launch (the reference's
// `layer_i_attention` is one task — /root/reference/test_gpt2.py:80-89, qkv + proj weights):
//
//   phase 1  qkv = LN(x) W_qkv'^T + b'          folded norm, row statistics handed over by x's
//                                              producer (ext_stats); 64 x 64 tiles: one tile =
//                                              one head's q, k or v columns for 64 rows
//   phase 2  o   = causal softmax(q k^T) v      one item = 64 queries of one (batch, head), 2 key
//                                              groups (attention_impl.h)
//   phase 3  out = o W_o^T + b_o + residual     64 x 64 tiles, 2 K groups; row statistics of out
//                                              for the next folded norm (stats_out)
//
// Work items are handed out by an agent-scope TICKET, not by blockIdx: a workgroup takes the next
// item when it starts, items are numbered phase by phase, so every item an item waits for has a
// smaller ticket and is already held by a running workgroup — progress is guaranteed whatever
// number of workgroups the chip (or a co-running kernel) leaves resident. Hand-offs follow the
// sc1 form of MI355X_MICROARCH.md's inter-workgroup visibility table (as gemm_fused.hip): the
// producer stores its tile write-through (sc1), drains (vmcnt 0), and one lane adds to an
// agent-scope counter; the consumer's lane 0 polls the counter, the workgroup barriers, and every
// load of produced bytes is an sc1 load (buffer loads / LDS-DMA with aux sc1).
//   qready[rb * n_head + h]: arrived q / k / v tiles of head h for 64-row block rb (3 = ready)
//   oready[qt]             : heads done for 64-row block qt (n_head = ready)
// Causality makes the hand-off fine-grained: query tile qt needs only row blocks 0..qt, so the
// light early query tiles start as soon as their rows exist. The last workgroup to finish resets
// every counter for the next launch. A poll past its spin bound sets the error word and proceeds
// (wrong numbers, never a hang).
#include <algorithm>
#include <cstdlib>

#include "attention_impl.h"
#include "gemm_glds_impl.h"

namespace {

// Every phase fits 64 KiB of LDS and 8 waves, so TWO workgroups share a CU and the whole grid
// (GPT-2: 288 + 96 + 96 = 480 items) is resident at once on 256 CUs — no item waits for a CU
// (v1, with 144 KiB phases and one workgroup per CU, dispatched the out-proj tiles only as
// attention items retired: profiles/r6_status/attn_block_stamps_v1.txt)
using P1 = Cfg<64, 64, 2, 2, 2, 0, 0, 2>;    // QKV (config 17): 512 x 2304 -> 8 x 36 = 288 tiles
using P3 = Cfg<64, 64, 2, 2, 2, 0, 0, 2>;    // out-proj (config 17): 512 x 768 -> 8 x 12 = 96 tiles
using AC = dls_attn::AttnCfg<64, 4, 2, 2>;   // 64 queries x 2 key groups of 64 keys per stage
constexpr int kThreads = 512;
static_assert(P1::T == kThreads && P3::T == kThreads && AC::NWT * 64 == kThreads, "one block size for all phases");
static_assert(P1::BN == 64 && AC::QB == P3::BM, "a q/k/v tile is one head's columns; an out tile one query tile");
constexpr int kLdsBytes = std::max({P1::LDS_UNITS * 16, P3::LDS_UNITS * 16, AC::SMEM});
constexpr int kHeadDim = 64;

struct Items {
  int n1, n2, n3, tiles_m1, tiles_m3, n_qt;
};

__device__ __forceinline__ Items items_of(const AttnBlockArgs& p) {
  Items it;
  it.tiles_m1 = p.M / P1::BM;
  it.n1 = it.tiles_m1 * (3 * p.H / P1::BN);
  it.n_qt = p.S / AC::QB;
  it.n2 = it.n_qt * p.n_head * p.B;
  it.tiles_m3 = p.M / P3::BM;
  it.n3 = it.tiles_m3 * (p.H / P3::BN);
  return it;
}

// counters sit on cache lines of their own (kPad ints apart): a poller hammers only its line
constexpr int kPad = 32;

// lane 0: spin until *ctr >= need (relaxed agent-scope loads, s_sleep between polls: every
// waiting workgroup polls, so a short sleep loads the L2 channel the producers publish through)
__device__ __forceinline__ void wait_count(const int* ctr, int need, const AttnBlockArgs& p) {
  int spins = 0;
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
    __builtin_amdgcn_s_sleep(8);
    if (++spins > p.spin_limit) {
      __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
}

// every wave's (write-through) stores drained, then ONE agent-scope arrival
__device__ __forceinline__ void publish(int* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// STAMP (diagnostic launches, p.stamps != null): per workgroup [item, start, wait done, end] in
// 100 MHz ticks (s_memrealtime), stored by thread 0 at the end
template <bool STAMP>
__global__ __launch_bounds__(kThreads) void attn_block_kernel(AttnBlockArgs p) {
  __shared__ __attribute__((aligned(16))) bf16x8 smem[kLdsBytes / 16];
  unsigned long long t_start = 0, t_wait = 0;
  if constexpr (STAMP) t_start = __builtin_amdgcn_s_memrealtime();
  __shared__ int s_item;
  int* ticket = p.sync;
  int* done = p.sync + kPad;
  const Items it = items_of(p);
  int* qready = p.sync + 2 * kPad;
  int* oready = qready + it.tiles_m1 * p.n_head * kPad;
  if (threadIdx.x == 0) s_item = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int item = s_item;
  const bf16* qkv = (const bf16*)p.qkv;

  if (item < it.n1) {
    // ---- phase 1: one q / k / v tile of the QKV GEMM (folded norm, ext row statistics)
    const int tm = item % it.tiles_m1, tn = item / it.tiles_m1;
    if constexpr (STAMP) t_wait = __builtin_amdgcn_s_memrealtime();
    const Epi ep{RopeArgs{}, nullptr, p.ext_stats, nullptr};
    glds_tile<P1, 0, 0, false, false, 0, true>(smem, (const bf16*)p.x, p.ldx, (const bf16*)p.w1, p.H,
                                               (bf16*)p.qkv, p.ldqkv, (const bf16*)p.b1, nullptr, 0, nullptr, p.M,
                                               p.M, 3 * p.H, p.H, 0, 1.0f, 0, p.H, tm, tn, p.colsum1, p.ln_mode,
                                               p.ln_eps, ep);
    const int head = (tn * P1::BN % p.H) / kHeadDim;
    publish(qready + (tm * p.n_head + head) * kPad);
  } else if (item < it.n1 + it.n2) {
    // ---- phase 2: 32 queries of one (batch, head); heaviest query tiles first
    const int j = item - it.n1;
    const int h = j % p.n_head, rest = j / p.n_head;
    const int qt = it.n_qt - 1 - rest % it.n_qt, b = rest / it.n_qt;
    if (threadIdx.x == 0) {
      const int row_lo = b * p.S, row_hi = b * p.S + (qt + 1) * AC::QB;  // keys 0..row_hi-1 (causal)
      for (int rb = row_lo / P1::BM; rb * P1::BM < row_hi; ++rb) wait_count(qready + (rb * p.n_head + h) * kPad, 3, p);
    }
    __syncthreads();  // the block's waves load q / k / v only after the poll has matched
    if constexpr (STAMP) t_wait = __builtin_amdgcn_s_memrealtime();
    const float sl2 = p.scale * 1.4426950408889634f;
    dls_attn::attn_item<kHeadDim, AC::NW, AC::ST, AC::KS, false, true>(
        reinterpret_cast<char*>(smem), qt, 0, 1, h, b, qkv, p.ldqkv, qkv + p.H, p.ldqkv, qkv + 2 * p.H, p.ldqkv,
        (bf16*)p.o, p.ldo, p.S, p.n_head, p.n_head, sl2, 1, it.n_qt, p.S, 0, /*flags: write-through*/ 1, nullptr,
        nullptr, 0);
    publish(oready + (b * it.n_qt + qt) * kPad);
  } else if (item < it.n1 + it.n2 + it.n3) {
    // ---- phase 3: one out-proj tile (+ bias + residual, next norm's row statistics)
    const int j = item - it.n1 - it.n2;
    const int tm = j % it.tiles_m3, tn = j / it.tiles_m3;
    if (threadIdx.x == 0) wait_count(oready + tm * kPad, p.n_head, p);
    __syncthreads();
    if constexpr (STAMP) t_wait = __builtin_amdgcn_s_memrealtime();
    const Epi ep{RopeArgs{}, p.stats_out, nullptr, nullptr};
    glds_tile<P3, 0, 0, false, false, kPolWT, false, kPolWT>(
        smem, (const bf16*)p.o, p.ldo, (const bf16*)p.wo, p.H, (bf16*)p.out, p.ldout, (const bf16*)p.bo,
        (const bf16*)p.R, p.ldr, nullptr, p.M, p.M, p.H, p.H, 0, 1.0f, 0, p.H, tm, tn, nullptr, 0, 0.f, ep);
  }
  // the last workgroup to finish resets every counter for the next launch (all others have
  // passed their polls and made their arrivals by then)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (STAMP) {
    if (threadIdx.x == 0) {
      unsigned long long* st = p.stamps + 4 * (size_t)blockIdx.x;
      st[0] = (unsigned long long)item;
      st[1] = t_start;
      st[2] = t_wait;
      st[3] = __builtin_amdgcn_s_memrealtime();
    }
  }
  if (threadIdx.x == 0) {
    const int total = it.n1 + it.n2 + it.n3;
    if (__hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1) {
      const int n = 2 + it.tiles_m1 * p.n_head + it.n_qt * p.B;
      for (int k = 0; k < n; ++k) __hip_atomic_store(p.sync + k * kPad, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

int attn_block_sync_ints(int M, int S, int B, int n_head) {
  return (2 + (M / P1::BM) * n_head + (S / AC::QB) * B) * kPad;
}

bool attn_block_supported(int M, int H, int B, int S, int n_head, int n_kv_head, int D) {
  return D == kHeadDim && n_kv_head == n_head && H == n_head * D && M == B * S && M % P1::BM == 0 &&
         S % AC::QB == 0 && H % (P1::BK * P1::KG) == 0 && H / (P1::BK * P1::KG) >= 2 && H % P3::BN == 0 &&
         H % (P3::BK * P3::KG) == 0 && H / (P3::BK * P3::KG) >= 2 && (3 * H) % P1::BN == 0;
}

void launch_attn_block(const AttnBlockArgs& p, hipStream_t s) {
  const int n1 = (p.M / P1::BM) * (3 * p.H / P1::BN);
  const int n2 = (p.S / AC::QB) * p.n_head * p.B;
  const int n3 = (p.M / P3::BM) * (p.H / P3::BN);
  if (p.stamps)
    hipLaunchKernelGGL(attn_block_kernel<true>, dim3(n1 + n2 + n3), dim3(kThreads), 0, s, p);
  else
    hipLaunchKernelGGL(attn_block_kernel<false>, dim3(n1 + n2 + n3), dim3(kThreads), 0, s, p);
}
