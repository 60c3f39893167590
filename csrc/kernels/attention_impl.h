// Flash-attention device code shared by the standalone kernel (attention.hip) and the one-launch
// attention block (attn_block.hip): one work item = QB queries of one (batch, head), walking its
// causal key range in KS key groups. See attention.hip for the formulation.
#pragma once
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

namespace dls_attn {

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

// SPLIT: every block takes ONE key tile (KTS keys) of one query tile — a query tile's key range
// is spread over as many blocks as it has tiles, so no CU streams a long causal row's whole K/V
// (the per-CU LDS-DMA intake bounds a stage); the blocks of a query tile publish their
// unnormalised (o, m, l) write-through into `part`, draw a ticket from cnt[query tile], and the
// last arriver merges the others' partials and stores the output (it resets the ticket)
template <int D, int NW, int ST, int KS, bool SPLIT, bool SC1>
__device__ __forceinline__ void attn_item(char* smem, int qt, int c, int nch, int h, int b, const bf16* __restrict__ Q,
                                          int ldq, const bf16* __restrict__ Kp, int ldk, const bf16* __restrict__ Vp,
                                          int ldv, bf16* __restrict__ O, int ldo, int S, int n_head, int n_kv_head,
                                          float scale_log2, int causal, int n_qtiles, int Sq, int q_off, int flags,
                                          float* __restrict__ part, int* __restrict__ cnt, int maxc) {
  using C = AttnCfg<D, NW, ST, KS>;
  constexpr int kDmaAux = SC1 ? 16 : 0;  // K/V DMA: sc1 when another workgroup of the launch wrote them
  const int tid = threadIdx.x, lane = tid & 63, wave_id = tid >> 6;
  // KS > 1: wave group hg takes keys [hg*64, hg*64+64) of every stage (the causal row's key
  // range is walked by KS independent online-softmax chains, merged through LDS at the end)
  const int wave = wave_id % NW, hg = wave_id / NW;
  const int g = lane >> 4, li = lane & 15;
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
    if constexpr (SC1) {
      // Q written by another workgroup of the same launch (attn_block.hip): sc1 loads, which
      // no stale line of this CU's L1 can serve
      const auto rq = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(Q), 0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int ks = 0; ks < C::NQK; ++ks) {
        const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(
            rq, (int)(((qtok0 + qrow) * ldq + h * D + 32 * ks + 8 * g) * 2), 0, 16);
        qf[ks] = *reinterpret_cast<const bf16x8*>(&u);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < C::NQK; ++ks)
        qf[ks] = *reinterpret_cast<const bf16x8*>(Q + (qtok0 + qrow) * ldq + h * D + 32 * ks + 8 * g);
    }
  }

  // LDS-DMA source pointers: instruction j of this wave -> operand (K or V) rows
  const int kv_end = causal ? min(S, q_off + qt * C::QB + C::QB) : S;
  const int ntiles = (kv_end + C::KTS - 1) / C::KTS;
  const int t0 = SPLIT ? c : 0, t1 = SPLIT ? c + 1 : ntiles;
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
    dptr[j] = dsrc[j] + (size_t)(drow[j] + t0 * C::KTS) * dstep[j];
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
                                       16, 0, kDmaAux);
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
    if (t0 + p < t1) issue(t0 + p);
  for (int t = t0; t < t1; ++t) {
    // tile t has landed once at most min(ST-2, tiles issued after t) tiles are in flight
    wait_tiles<C::PW, ST - 2>(min(ST - 2, t1 - 1 - t));
    raw_barrier();
    if (t == t0) {
      DLS_ASTAMP(1)
    }
    if (t + ST - 1 < t1) issue(t + ST - 1);  // into the buffer everyone finished in t-1
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
    if (hg == 0) {
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
  }
  if constexpr (SPLIT) {
    if (nch > 1) {
      // publish this chunk's (o, m, l) per lane of key group 0: REC2 floats, o then (m, l)
      constexpr int REC2 = C::ND * 4 + 4;
      constexpr int LN = C::NW * 64;
      const int me = wave * 64 + lane;
      const size_t tile_id = ((size_t)b * n_head + h) * n_qtiles + qt;
      float* pp = part + tile_id * (size_t)maxc * LN * REC2;
      const auto rp = __builtin_amdgcn_make_buffer_rsrc(pp, 0, 0x7fffffff, 0x00020000);
      if (hg == 0) {
        const int base = ((c * LN + me) * REC2) * 4;
#pragma unroll
        for (int dn = 0; dn < C::ND; ++dn)
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{__float_as_uint(o[dn][0]), __float_as_uint(o[dn][1]), __float_as_uint(o[dn][2]),
                    __float_as_uint(o[dn][3])},
              rp, base + dn * 16, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(m_run), __float_as_uint(l_run)}, rp,
                                              base + C::ND * 16, 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's write-through stores landed
      __syncthreads();
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(cnt + tile_id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == nch - 1;
        if (last) __hip_atomic_store(cnt + tile_id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
        flag[0] = last;
      }
      __syncthreads();
      if (!flag[0] || hg != 0) return;  // block-uniform, then key group 0 only
      // the last arriver merges every other chunk of its query tile (sc1 loads: no stale copy)
      for (int c2 = 0; c2 < nch; ++c2) {
        if (c2 == c) continue;
        const int base = ((c2 * LN + me) * REC2) * 4;
        f32x4 o2[C::ND];
#pragma unroll
        for (int dn = 0; dn < C::ND; ++dn) {
          const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rp, base + dn * 16, 0, 16);
          o2[dn] = f32x4{__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3])};
        }
        const u32x2 ml = __builtin_amdgcn_raw_buffer_load_b64(rp, base + C::ND * 16, 0, 16);
        const float m2 = __uint_as_float(ml[0]), l2 = __uint_as_float(ml[1]);
        const float mm = fmaxf(fmaxf(m_run, m2), -1e30f);
        const float a0 = __builtin_amdgcn_exp2f((m_run - mm) * scale_log2);
        const float a1 = __builtin_amdgcn_exp2f((m2 - mm) * scale_log2);
        l_run = l_run * a0 + l2 * a1;
        m_run = mm;
#pragma unroll
        for (int dn = 0; dn < C::ND; ++dn) o[dn] = o[dn] * a0 + o2[dn] * a1;
      }
    }
  }
  if (hg != 0) return;
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

}  // namespace dls_attn
