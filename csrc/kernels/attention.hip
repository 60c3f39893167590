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
#include "common.h"
#include "kernels.h"

// Phase stamps for a diagnostic build (benchmarks/attn_stamps.hip defines DLS_ASTAMP to read the
// 100 MHz clock into a register; the block's wave 0 stores them once at the very end, so no
// extra memory operation joins the counted vmcnt waits). Compiled out otherwise.
#ifndef DLS_ASTAMP
#define DLS_ASTAMP_DECL()
#define DLS_ASTAMP(k)
#define DLS_ASTAMP_STORE()
#endif

namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

template <bool B>
struct BoolC {
  static constexpr bool value = B;
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }
// wait until at most `ahead` tiles (PW DMA instructions each) are still in flight
template <int PW, int A>
__device__ __forceinline__ void wait_tiles(int ahead) {
  if constexpr (A <= 0) {
    wait_vm<0>();
  } else {
    if (ahead >= A) wait_vm<PW * A>();
    else wait_tiles<PW, A - 1>(ahead);
  }
}

template <int D, int NW_, int ST_ = 2, int KS_ = 1>
struct AttnCfg {
  static constexpr int NW = NW_;                 // query waves per block (16 queries each)
  static constexpr int KS = KS_;                 // key halves per stage: KS wave groups split each stage's keys
  static constexpr int NWT = NW * KS;            // waves per block
  static constexpr int ST = ST_;                 // K/V stages (ST-1 tiles in flight)
  static constexpr int QB = 16 * NW;             // queries per block
  static constexpr int KT = 64;                  // keys per wave per stage
  static constexpr int KTS = KT * KS;            // keys per stage
  static constexpr int RB = D * 2;               // bytes per K/V row
  static constexpr int CH = D / 8;               // 16-B chunks per row
  static constexpr int ROWS_PER_INSTR = 1024 / RB;
  static constexpr int INSTR = KTS / ROWS_PER_INSTR;  // per operand per stage
  static constexpr int PW = 2 * INSTR / NWT;          // per wave per stage (K and V)
  static constexpr int TILE_BYTES = KTS * RB;         // one operand
  static constexpr int BUF_BYTES = 2 * TILE_BYTES;    // K + V
  static constexpr int NQK = D / 32;                  // k-steps of S^T
  static constexpr int ND = D / 16;                   // output d-subtiles
  static constexpr int MERGE_BYTES = KS > 1 ? (KS - 1) * NW * 64 * (ND * 4 + 2) * 4 : 0;
  static constexpr int SMEM = ST * BUF_BYTES > MERGE_BYTES ? ST * BUF_BYTES : MERGE_BYTES;
  static_assert(PW * (ST - 2) <= 63 && PW * NWT == 2 * INSTR, "DMA split");
  static_assert(SMEM <= 163840, "LDS budget");
};

__device__ __forceinline__ int swz(int row, int ch_mask) { return row & ch_mask; }

// Cross-lane reduction steps on the VALU (v_permlane16/32_swap, CDNA4) instead of
// ds_bpermute: with the same value in both operands the two results are x[l] and x[l ^ 16]
// (resp. ^ 32) in some order, so their max / sum is one butterfly step.
template <bool MAX, int DIST>
__device__ __forceinline__ float xlane(float x) {
  const unsigned u = __float_as_uint(x);
  float a, b;
  if constexpr (DIST == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
  }
  return MAX ? fmaxf(a, b) : a + b;
}

template <int D, int NW, int ST, int KS>
__global__ __launch_bounds__(64 * NW * KS) void attn_fwd_kernel(const bf16* __restrict__ Q, int ldq,
                                                       const bf16* __restrict__ Kp, int ldk,
                                                       const bf16* __restrict__ Vp, int ldv, bf16* __restrict__ O,
                                                       int ldo, int S, int n_head, int n_kv_head, float scale_log2,
                                                       int causal, int n_qtiles, int Sq, int q_off, int flags) {
  using C = AttnCfg<D, NW, ST, KS>;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave_id = tid >> 6;
  // KS > 1: wave group hg takes keys [hg*64, hg*64+64) of every stage (the causal row's key
  // range is walked by KS independent online-softmax chains, merged through LDS at the end)
  const int wave = wave_id % NW, hg = wave_id / NW;
  const int g = lane >> 4, li = lane & 15;
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
  const int qt = causal ? (n_qtiles - 1 - bx) : bx;  // heaviest first
  DLS_ASTAMP_DECL()
  DLS_ASTAMP(0)
  const int kvh = h / (n_head / n_kv_head);
  const int q0 = qt * C::QB + wave * 16;  // this wave's 16 queries (local rows of the q chunk)
  const size_t tok0 = (size_t)b * S;       // first key row of this batch
  const size_t qtok0 = (size_t)b * Sq;     // first query / output row of this batch

  // Q^T as the B operand: lane holds Q[q0 + li][32*ks + 8*g + j]
  bf16x8 qf[C::NQK];
  {
    const int qrow = min(q0 + li, Sq - 1);
#pragma unroll
    for (int ks = 0; ks < C::NQK; ++ks)
      qf[ks] = *reinterpret_cast<const bf16x8*>(Q + (qtok0 + qrow) * ldq + h * D + 32 * ks + 8 * g);
  }

  // LDS-DMA source pointers: instruction j of this wave -> operand (K or V) rows
  const int kv_end = causal ? min(S, q_off + qt * C::QB + C::QB) : S;
  const int ntiles = (kv_end + C::KTS - 1) / C::KTS;
  // per-lane DMA sources, computed once: instruction j of this wave covers operand op's
  // rows r0..r0+ROWS_PER_INSTR-1 of every tile; a tile only moves the base by KT rows.
  // Rows past S (the last tile) are clamped to S-1 (their scores are masked to -inf).
  const bf16* dsrc[C::PW];
  int drow[C::PW], doff[C::PW];
  size_t dstep[C::PW];
#pragma unroll
  for (int j = 0; j < C::PW; ++j) {
    const int ins = wave_id * C::PW + j;         // 0 .. 2*INSTR-1
    const int op = ins / C::INSTR;               // 0 = K, 1 = V
    const int r0 = (ins % C::INSTR) * C::ROWS_PER_INSTR;
    const int row = r0 + lane / C::CH;
    const int gch = (lane % C::CH) ^ swz(row, C::CH - 1);
    const int ld = op == 0 ? ldk : ldv;
    dsrc[j] = (op == 0 ? Kp : Vp) + tok0 * ld + kvh * D + gch * 8;
    dstep[j] = (size_t)ld;
    drow[j] = row;
    doff[j] = op * C::TILE_BYTES + r0 * C::RB;
  }
  const bool tail_clamp = (S % C::KTS) != 0;
  // running per-lane sources: issue() is called for t = 0, 1, 2, ... in order and moves each
  // pointer one tile (KTS rows) on — no per-tile 64-bit address arithmetic (the ragged last
  // tile clamps its rows explicitly)
  const bf16* dptr[C::PW];
  size_t dinc[C::PW];
#pragma unroll
  for (int j = 0; j < C::PW; ++j) {
    dptr[j] = dsrc[j] + (size_t)drow[j] * dstep[j];
    dinc[j] = (size_t)C::KTS * dstep[j];
  }
  auto issue = [&](int t) {
    char* buf = smem + (t % ST) * C::BUF_BYTES;
    const bool clamp = tail_clamp && (t + 1) * C::KTS > S;
#pragma unroll
    for (int j = 0; j < C::PW; ++j) {
      const bf16* src = dptr[j];
      if (clamp) src = dsrc[j] + (size_t)min(t * C::KTS + drow[j], S - 1) * dstep[j];
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(buf + doff[j]),
                                       16, 0, 0);
      dptr[j] += dinc[j];
    }
  };

  f32x4 o[C::ND];
#pragma unroll
  for (int i = 0; i < C::ND; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;  // for query q0 + li (replicated over the 4 lane groups)
  const int my_q = q0 + li;         // local query row
  const int gq = q_off + my_q;       // its global position (causal mask)

  // one 64-key stage of this wave's chain: S^T = K Q^T, online softmax, O^T += V^T P^T
  auto stage = [&](int t, int key0, auto mask_c) {
    const char* kb = smem + (t % ST) * C::BUF_BYTES + hg * C::KT * C::RB;
    const char* vb = kb + C::TILE_BYTES;
    // ---- S^T = K Q^T : 4 key-subtiles x 16 queries
    f32x4 s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = 16 * n + li;
#pragma unroll
      for (int ks = 0; ks < C::NQK; ++ks) {
        const int c = 4 * ks + g;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + row * C::RB + ((c ^ swz(row, C::CH - 1)) << 4));
        s[n] = mfma16x16x32(kf, qf[ks], s[n]);
      }
    }
    // ---- online softmax for query my_q; scores s[n][i] <-> key key0 + 16n + 4g + i.
    // Raw scores are kept; the scale is folded into the exponent: p = 2^(s*c - m*c).
    if constexpr (decltype(mask_c)::value) {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = key0 + 16 * n + 4 * g + i;
          if (key >= S || (causal && key > gq)) s[n][i] = -INFINITY;
        }
    }
    float mx = fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3]));
#pragma unroll
    for (int n = 1; n < 4; ++n) mx = fmaxf(mx, fmaxf(fmaxf(s[n][0], s[n][1]), fmaxf(s[n][2], s[n][3])));
    mx = xlane<true, 16>(mx);
    mx = xlane<true, 32>(mx);
    // m_new is finite from the first tile on (key 0 is visible to every query); the clamp
    // only keeps -inf - -inf out of padded rows
    const float m_new = fmaxf(fmaxf(m_run, mx), -1e30f);
    const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * scale_log2);
    const float mc = m_new * scale_log2;
    float sum = 0.f;
    bf16x8 pf[2];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __builtin_amdgcn_exp2f(fmaf(s[n][i], scale_log2, -mc));
        sum += e;
        pf[n >> 1][4 * (n & 1) + i] = f2bf(e);
      }
    sum = xlane<false, 16>(sum);
    sum = xlane<false, 32>(sum);
    l_run = l_run * alpha + sum;
    m_run = m_new;
#pragma unroll
    for (int dn = 0; dn < C::ND; ++dn) o[dn] *= alpha;

    // ---- O^T += V^T P^T ; V^T fragment element j <-> key 32ks + 16(j>>2) + 4g + (j&3)
    const int q4 = li >> 2, p4 = li & 3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int dn = 0; dn < C::ND; ++dn) {
        const int c = 2 * dn + (p4 >> 1);
        const int row0 = 32 * ks + 4 * g + q4;
        const int row1 = row0 + 16;
        const lds_bf16x4* a0 = (const lds_bf16x4*)(vb + row0 * C::RB + ((c ^ swz(row0, C::CH - 1)) << 4) + (p4 & 1) * 8);
        const lds_bf16x4* a1 = (const lds_bf16x4*)(vb + row1 * C::RB + ((c ^ swz(row1, C::CH - 1)) << 4) + (p4 & 1) * 8);
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
        const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[dn] = mfma16x16x32(vf, pf[ks], o[dn]);
      }
    }
  };

#pragma unroll
  for (int p = 0; p < ST - 1; ++p)
    if (p < ntiles) issue(p);
  for (int t = 0; t < ntiles; ++t) {
    // tile t has landed once at most min(ST-2, tiles issued after t) tiles are in flight
    wait_tiles<C::PW, ST - 2>(min(ST - 2, ntiles - 1 - t));
    raw_barrier();
    if (t == 0) {
      DLS_ASTAMP(1)
    }
    if (t + ST - 1 < ntiles) issue(t + ST - 1);  // into the buffer everyone finished in t-1
    const int key0 = t * C::KTS + hg * C::KT;
    // Masks only on the wave's diagonal tile and the ragged last tile: a wave-uniform choice
    // between two instantiations of the stage (a plain branch was if-converted, so every tile
    // paid for the mask compares and selects)
    const bool masked = (key0 + C::KT > S) || (causal && key0 + C::KT - 1 > q_off + q0);
    if (masked) stage(t, key0, BoolC<true>{});
    else stage(t, key0, BoolC<false>{});
  }
  DLS_ASTAMP(2)
  if constexpr (KS > 1) {
    // merge the key-group chains in ONE exchange: every group hg > 0 publishes (o, m, l) into
    // its own LDS slab at once (field-major: a wave's 64 lanes store 64 consecutive floats, no
    // bank conflicts), one barrier, and group 0 rescales and sums all of them in registers
    __syncthreads();  // all DMA landed and every wave is done with the K/V buffers
    float* mg = reinterpret_cast<float*>(smem);
    constexpr int REC = C::ND * 4 + 2;  // floats per lane: o, m, l
    constexpr int LN = C::NW * 64;      // lanes of one key group
    const int me = wave * 64 + lane;
    if (hg > 0) {
      float* r = mg + (hg - 1) * REC * LN + me;
#pragma unroll
      for (int dn = 0; dn < C::ND; ++dn)
#pragma unroll
        for (int i = 0; i < 4; ++i) r[(dn * 4 + i) * LN] = o[dn][i];
      r[C::ND * 4 * LN] = m_run;
      r[(C::ND * 4 + 1) * LN] = l_run;
    }
    __syncthreads();
    if (hg != 0) return;
    float mo[KS - 1], lo_[KS - 1];
    float mm = m_run;
#pragma unroll
    for (int h2 = 0; h2 < KS - 1; ++h2) {
      const float* r = mg + h2 * REC * LN + me;
      mo[h2] = r[C::ND * 4 * LN];
      lo_[h2] = r[(C::ND * 4 + 1) * LN];
      mm = fmaxf(mm, mo[h2]);
    }
    mm = fmaxf(mm, -1e30f);
    const float a0 = __builtin_amdgcn_exp2f((m_run - mm) * scale_log2);
    l_run *= a0;
#pragma unroll
    for (int dn = 0; dn < C::ND; ++dn) o[dn] *= a0;
#pragma unroll
    for (int h2 = 0; h2 < KS - 1; ++h2) {
      const float* r = mg + h2 * REC * LN + me;
      const float a1 = __builtin_amdgcn_exp2f((mo[h2] - mm) * scale_log2);
      l_run += lo_[h2] * a1;
#pragma unroll
      for (int dn = 0; dn < C::ND; ++dn)
#pragma unroll
        for (int i = 0; i < 4; ++i) o[dn][i] += r[(dn * 4 + i) * LN] * a1;
    }
    m_run = mm;
  }
  DLS_ASTAMP(3)
  // ---- normalise and store O[q][d]: lane holds d = 16dn + 4g + i for query my_q
  if (my_q < Sq) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    bf16* orow = O + (qtok0 + my_q) * ldo + h * D;
    // wt: write-through (sc1) stores — the tile leaves the XCD's L2 as it is written, so the
    // kernel boundary has no dirty lines of it to write back (AttnArgs::flags bit 0)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(O, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int dn = 0; dn < C::ND; ++dn) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(o[dn][i] * inv);
      if (flags & 1)
        __builtin_amdgcn_raw_buffer_store_b64(*reinterpret_cast<const u32x2*>(&v), rs,
                                              (int)(((qtok0 + my_q) * ldo + h * D + 16 * dn + 4 * g) * 2), 0, 16);
      else
        *reinterpret_cast<bf16x4*>(orow + 16 * dn + 4 * g) = v;
    }
  }
  DLS_ASTAMP(4)
  DLS_ASTAMP_STORE()
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
                     a.Sq > 0 ? a.q_off : 0, a.flags);
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

void launch_attention_fwd(const AttnArgs& a, hipStream_t s) {
  if (a.D == 64) launch_variant<64>(a, a.variant, s);
  else launch_variant<128>(a, a.variant, s);
}
