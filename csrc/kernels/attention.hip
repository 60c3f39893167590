// Flash attention forward on MFMA (causal or full, MHA or GQA), bf16 in/out — v2.
//
// Workgroup = 64 queries of one (batch, head): 4 waves x 16 queries; 64-key tiles.
// Swapped-operand formulation (cdna_hip_programming.md §3 "accumulator tile as the
// next MFMA's operand", T10, T12 idea without the permlanes):
//   S^T = K Q^T    A = K rows straight from LDS (16-B reads), B = Q^T from registers.
//                  Each lane then holds 16 scores of ONE query -> the online-softmax max and
//                  sum need 2 cross-lane shuffles (xor 16, 32) instead of a 16-lane tree.
//   O^T += V^T P^T B = P^T is taken from the S^T accumulators IN PLACE (no LDS round
//                  trip): the MFMA's k order is permuted identically on both operands
//                  (element j of lane group g <-> key 16*(j>>2) + 4g + (j&3)), and the
//                  matching V^T fragment is two ds_read_b64_tr_b16 transposed reads of the
//                  row-major V tile.
// K/V tiles arrive by LDS-DMA (global_load_lds_dwordx4; XOR chunk swizzle applied to the
// per-lane source address, rule 21), double-buffered: wait(tile t) -> ONE barrier ->
// issue(tile t+1 into the buffer everyone finished in t-1) -> compute t.
// Causal blocks stop at the diagonal tile and are launched heaviest-first.
#include <algorithm>

#include "common.h"
#include "kernels.h"

#include "attention_impl.h"

namespace {

using dls_attn::AttnCfg;

template <int D, int NW, int ST, int KS, bool SPLIT = false>
__global__ __launch_bounds__(64 * NW * KS) void attn_fwd_kernel(const bf16* __restrict__ Q, int ldq,
                                                       const bf16* __restrict__ Kp, int ldk,
                                                       const bf16* __restrict__ Vp, int ldv, bf16* __restrict__ O,
                                                       int ldo, int S, int n_head, int n_kv_head, float scale_log2,
                                                       int causal, int n_qtiles, int Sq, int q_off, int flags,
                                                       float* __restrict__ part, int* __restrict__ cnt, int maxc) {
  using C = AttnCfg<D, NW, ST, KS>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  // flags bit 1: XCD-grouped blocks — the blocks of one (batch, head) run on one XCD (block
  // b goes to XCD b % 8; xcd_remap hands each XCD a contiguous range of logical blocks, query
  // tiles fastest), so the head's K/V rows come into ONE XCD's L2 from the MALL instead of all
  // eight; the heaviest-first order then holds within each XCD's range
  int bx = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  if (flags & 2) {
    const int lin = bx + gridDim.x * (h + gridDim.y * b);
    const int L = xcd_remap(lin, gridDim.x * gridDim.y * gridDim.z);
    bx = L % gridDim.x;
    h = (L / gridDim.x) % gridDim.y;
    b = L / (gridDim.x * gridDim.y);
  }
  // key tiles [t0, t1) of query tile qt (SPLIT: one tile, chunk c of nch)
  int qt, c = 0, nch = 1;
  if constexpr (SPLIT) {
    int rem = bx;
    qt = n_qtiles - 1;
    for (;;) {  // heaviest query tiles first; every block finds its item (bx < total items)
      const int kvq = causal ? min(S, q_off + qt * C::QB + C::QB) : S;
      nch = (kvq + C::KTS - 1) / C::KTS;
      if (rem < nch || qt == 0) break;
      rem -= nch;
      --qt;
    }
    c = min(rem, nch - 1);
  } else {
    qt = causal ? (n_qtiles - 1 - bx) : bx;  // heaviest first
  }
  dls_attn::attn_item<D, NW, ST, KS, SPLIT, false>(smem, qt, c, nch, h, b, Q, ldq, Kp, ldk, Vp, ldv, O, ldo, S, n_head,
                                                   n_kv_head, scale_log2, causal, n_qtiles, Sq, q_off, flags, part,
                                                   cnt, maxc);
}

}  // namespace

template <int D, int NW, int ST, int KS = 1>
static void launch_attn(const AttnArgs& a, hipStream_t s) {
  const int Sq = a.Sq > 0 ? a.Sq : a.S;
  const int nq = (Sq + 16 * NW - 1) / (16 * NW);
  dim3 grid(nq, a.n_head, a.B), block(64 * NW * KS);
  const float sl2 = a.scale * 1.4426950408889634f;
  hipLaunchKernelGGL((attn_fwd_kernel<D, NW, ST, KS>), grid, block, 0, s, static_cast<const bf16*>(a.q), a.ldq,
                     static_cast<const bf16*>(a.k), a.ldk, static_cast<const bf16*>(a.v), a.ldv,
                     static_cast<bf16*>(a.o), a.ldo, a.S, a.n_head, a.n_kv_head, sl2, a.causal, nq, Sq,
                     a.Sq > 0 ? a.q_off : 0, a.flags, nullptr, nullptr, 0);
}

// SPLIT launch: one block per (query tile, key tile) item; a.part / a.cnt from the caller
// (attention_split_sizes)
template <int D, int NW, int ST, int KS>
static void launch_attn_split(const AttnArgs& a, hipStream_t s) {
  using C = AttnCfg<D, NW, ST, KS>;
  const int Sq = a.Sq > 0 ? a.Sq : a.S, q_off = a.Sq > 0 ? a.q_off : 0;
  const int nq = (Sq + C::QB - 1) / C::QB;
  int items = 0;
  for (int qt = 0; qt < nq; ++qt) {
    const int kvq = a.causal ? std::min(a.S, q_off + qt * C::QB + C::QB) : a.S;
    items += (kvq + C::KTS - 1) / C::KTS;
  }
  dim3 grid(items, a.n_head, a.B), block(64 * NW * KS);
  const float sl2 = a.scale * 1.4426950408889634f;
  hipLaunchKernelGGL((attn_fwd_kernel<D, NW, ST, KS, true>), grid, block, 0, s, static_cast<const bf16*>(a.q),
                     a.ldq, static_cast<const bf16*>(a.k), a.ldk, static_cast<const bf16*>(a.v), a.ldv,
                     static_cast<bf16*>(a.o), a.ldo, a.S, a.n_head, a.n_kv_head, sl2, a.causal, nq, Sq, q_off,
                     a.flags & 1, static_cast<float*>(a.part), static_cast<int*>(a.cnt), (a.S + C::KTS - 1) / C::KTS);
}

template <int D>
static void launch_variant(const AttnArgs& a, int v, hipStream_t s) {
  switch (v) {
    case 1: launch_attn<D, 2, 2>(a, s); break;
    case 2: launch_attn<D, 4, 2>(a, s); break;
    case 3: launch_attn<D, 2, 3>(a, s); break;
    case 4: launch_attn<D, 4, 3>(a, s); break;
    // deep K/V rings: a causal row's whole key range (S=512, D=64) in flight at once
    case 5: launch_attn<D, 4, 4>(a, s); break;
    case 6: launch_attn<D, 4, (D == 64 ? 8 : 5)>(a, s); break;
    case 7: launch_attn<D, 2, (D == 64 ? 8 : 5)>(a, s); break;
    // key-split stages: two online-softmax chains per query group (shorter dependent chain
    // per wave, two waves per SIMD) merged in LDS
    case 8: launch_attn<D, 4, 2, 2>(a, s); break;
    case 9: launch_attn<D, 2, 2, 2>(a, s); break;
    case 10: launch_attn<D, 2, (D == 64 ? 3 : 2), 2>(a, s); break;
    case 11: launch_attn<D, 1, (D == 64 ? 4 : 2), 2>(a, s); break;
    // four key chains per query group (D = 128: two, the LDS holds no more)
    case 12: launch_attn<D, 1, 2, (D == 64 ? 4 : 2)>(a, s); break;
    case 13: launch_attn<D, 2, 2, (D == 64 ? 4 : 2)>(a, s); break;
    // one key tile per block, query tiles merged by their last arriver (needs a.part / a.cnt)
    case 14: launch_attn_split<D, 2, 2, 2>(a, s); break;
    default: {
      // 64-query blocks, 2 K/V stages fill the chip from ~320 blocks on (batch 8, S=2048);
      // below that the causal row's dependent chain is the kernel time, so split each stage's
      // keys over two wave groups (GPT-2 S=512: 96 blocks, 8.2 -> 6.2 us with 32-query blocks;
      // Llama-3-8B S=512: 256 blocks, 13.1 -> 11.9 us)
      const long blocks = (long)(((a.Sq > 0 ? a.Sq : a.S) + 63) / 64) * a.n_head * a.B;
      // (<= 128 blocks: four key groups per stage for D = 64 since the key-group merge is one
      // LDS exchange — GPT-2 S=512: 0.623 vs 0.629 ms per step, profiles/r4_ab/attention_merge.txt)
      if (blocks <= 128) launch_attn<D, 2, 2, (D == 64 ? 4 : 2)>(a, s);
      else if (blocks <= 320) launch_attn<D, 4, 2, 2>(a, s);
      else launch_attn<D, 4, 2>(a, s);
    }
  }
}

// workspace of the split variant (14): partial floats and ticket counters
void attention_split_sizes(const AttnArgs& a, size_t* part_floats, size_t* counters) {
  const int D = a.D, KTS = 128, QB = 32;  // launch_attn_split<D, 2, 2, 2>: 2 x 64 keys, 2 x 16 queries
  const int Sq = a.Sq > 0 ? a.Sq : a.S;
  const size_t nq = (Sq + QB - 1) / QB, maxc = (a.S + KTS - 1) / KTS;
  *counters = (size_t)a.B * a.n_head * nq;
  *part_floats = *counters * maxc * 128 * (D / 16 * 4 + 4);
}

void launch_attention_fwd(const AttnArgs& a, hipStream_t s) {
  if (a.D == 64) launch_variant<64>(a, a.variant, s);
  else launch_variant<128>(a, a.variant, s);
}
