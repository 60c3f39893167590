// gemm_glds_impl.h: the LDS-DMA GEMM's device code and per-config launcher, included by the
// per-config translation units gemm_glds_cfg*.hip (compiled in parallel) — see gemm_glds.hip.
#pragma once
// Multistage bf16 GEMM with LDS-DMA staging (global_load_lds_dwordx4), optional split-K.
//
//   C = act(alpha * A @ W^T + bias) + R      A [M][K], W [N][K] (K contiguous), K % 64 == 0
//
// Why this structure (cdna_hip_programming.md §5 "Pipelining across barriers", T1, T2):
//  * GPT-2 / Llama serving GEMMs have M = 512 rows: a grid barely covers the 256 CUs, so
//    each CU runs ~1 block and a K-loop that keeps ONE tile in flight is latency-bound —
//    especially when the weights stream cold from HBM (measured 1.6-2x slower inside the
//    DAG than in a hot-cache loop). Here STAGES-1 K-tiles are in flight per block.
//  * LDS-DMA needs no staging VGPRs and no ds_write pass; the image is lane-linear (1 KiB
//    per wave instruction = 8 rows x 128 B), so the XOR swizzle (chunk ^ (row & 7)) is
//    applied to the per-lane SOURCE address and again on the ds_read (rule 21).
//  * ONE raw s_barrier per K-tile: wait(tile kt) -> barrier -> issue(tile kt+STAGES-1 into
//    the buffer everyone finished reading before this barrier) -> MFMAs on tile kt. The
//    wait is a counted vmcnt (never 0 in steady state); __syncthreads() is avoided because
//    its fence drains every outstanding DMA.
//  * Split-K (host-chosen) multiplies the block count for skinny N; partial fp32 tiles go
//    to a workspace slab and a vectorised reduce kernel applies the fused epilogue.
//  * XCD-aware tile order (T1): the blocks of one weight panel share an XCD's L2.
#include <cstdlib>
#include <type_traits>
#include "common.h"
#include "kernels.h"
#include "gemm_glds_cfgs.h"

// In-kernel phase stamps for diagnostic builds (benchmarks/gemm_stamps.hip defines it before
// including this file); empty in the library.
#ifndef DLS_STAMP
#define DLS_STAMP(k)
#endif

namespace {

__device__ __forceinline__ int kslice_count(int K, int kslice) { return K / kslice; }

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most `ahead` tiles (PW DMA instructions each) are still in flight; the
// immediate must be a compile-time constant, so unroll over the possible values
template <int PW, int A>
__device__ __forceinline__ void wait_tiles(int ahead) {
  if constexpr (A == 0) {
    wait_vm<0>();
  } else {
    if (ahead >= A) wait_vm<PW * A>();
    else wait_tiles<PW, A - 1>(ahead);
  }
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

// BXS = extra weight (B) stages: 0 -> A and W tiles share STAGES buffers and travel
// together; >= 1 -> A keeps STAGES buffers (it is L2-resident: short latency) while the COLD
// weight stream gets STAGES + BXS, i.e. BXS more tiles of HBM latency covered inside the same
// 160 KiB of LDS (e.g. 256x256: 2 x 32 KiB A + 3 x 32 KiB W).
// KG_ = K groups: KG wave groups of WM x WN waves share each output tile; a stage holds KG
// consecutive 64-deep K-tiles and group g multiplies tile g of every stage (intra-block
// split-K: KG x the waves — and DMA issuers — per CU on a skinny grid, no reduce kernel; the
// groups' accumulators are summed through LDS before the epilogue).
// RING_ = 1: the 256x256 half-tile ring main loop (mainloop_ring) instead of whole-K-tile stages
// OCC_: waves per SIMD the kernel must allow (__launch_bounds__' second argument): 2 for the
// 4-wave tiles meant to run two workgroups per CU (at most 256 VGPRs + AGPRs per wave)
template <int BM_, int BN_, int WM_, int WN_, int STAGES_, int PRIO_ = 0, int BXS_ = 0, int KG_ = 1, int RING_ = 0,
          int OCC_ = 1>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, STAGES = STAGES_, PRIO = PRIO_, BXS = BXS_;
  static constexpr int KG = KG_, RING = RING_, OCC = OCC_;
  static constexpr int BK = 64, CH = 8;
  static constexpr int NW = WM * WN, T = 64 * NW * KG;
  static constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  // fragments of one 32-deep K half at a time (instead of both halves before the first MFMA)
  // for wave tiles with many fragments (32 x 224)
  static constexpr bool HALF_FRAGS = FM + FN > 12;
  // DMA instructions (8 rows x 128 B each) per wave: when the rows do not split evenly over
  // the waves, the last waves repeat the stage's last instruction (same bytes to the same LDS
  // slot), so every wave issues the same count and the counted vmcnt waits stay uniform
  static constexpr int ROWS = BM + BN, INSTR = ROWS / 8, PW = (INSTR + NW - 1) / NW;
  static constexpr int SUB = ROWS * CH;     // one 64-deep K-tile image (bf16x8 units)
  static constexpr int STAGE = SUB * KG;    // bf16x8 units
  // split staging (BXS > 0): separate A / W rings
  static constexpr int SA = STAGES, SB = STAGES + BXS;
  static constexpr int PWA = (BM / 8 + NW - 1) / NW, PWB = (BN / 8 + NW - 1) / NW;
  static constexpr bool EVEN = INSTR % NW == 0, EVEN_A = (BM / 8) % NW == 0, EVEN_B = (BN / 8) % NW == 0;
  static constexpr int A_STAGE = BM * CH, B_STAGE = BN * CH;
  static constexpr int LDS_UNITS = BXS ? SA * A_STAGE + SB * B_STAGE : STAGES * STAGE;
  static_assert(BM % 8 == 0 && BN % 8 == 0, "DMA pieces are 8 rows");
  static_assert(FM >= 1 && FN >= 1, "wave tile too small");
  static_assert(PW * (STAGES - 2) <= 63, "vmcnt range");
  static_assert(!BXS || (SA - 2) * PWA + (SA - 1) * PWB <= 63, "vmcnt range (split rings)");
  static_assert(STAGES >= 2 && STAGES <= 8, "stages");
  static_assert(LDS_UNITS * 16 <= 163840, "LDS budget");
  static_assert(KG == 1 || (BXS == 0 && PRIO == 0), "K groups use the joint ring");
  static_assert(KG == 1 || NW * 64 * FM * FN * 16 <= LDS_UNITS * 16, "K-group reduction must fit the LDS");
  static_assert(!RING || (BM == 256 && BN == 256 && WM == 2 && WN == 4 && STAGES == 2 && KG == 1 && BXS == 0),
                "the ring main loop is written for 256x256 tiles, 8 waves as 2 x 4, 8 x 16 KiB slots");
};

// split rings with a W ring D = BXS tiles deeper than the A ring: wait until at most
// a*PWA + b*PWB DMA instructions are outstanding, a in [0, AM], b in [0, BM] (any pair)
template <int PWA, int PWB, int AM, int BM>
__device__ __forceinline__ void wait_ab_any(int a, int b) {
  if constexpr (AM > 0) {
    if (a < AM) {
      wait_ab_any<PWA, PWB, AM - 1, BM>(a, b);
      return;
    }
  }
  if constexpr (BM > 0) {
    if (b < BM) {
      wait_ab_any<PWA, PWB, AM, BM - 1>(a, b);
      return;
    }
  }
  wait_vm<AM * PWA + BM * PWB>();
}
// split rings: wait until at most a*PWA + b*PWB DMA instructions are outstanding, with
// a in [0, AMAX] and b in {a, a + 1} (see the issue order in glds_tile)
template <int PWA, int PWB, int A>
__device__ __forceinline__ void wait_ab(int a, int b) {
  if constexpr (A == 0) {
    if (b >= 1) wait_vm<PWB>();
    else wait_vm<0>();
  } else {
    if (a >= A) {
      if (b > A) wait_vm<A * PWA + (A + 1) * PWB>();
      else wait_vm<A * PWA + A * PWB>();
    } else {
      wait_ab<PWA, PWB, A - 1>(a, b);
    }
  }
}

// MFMAs of one staged K-tile: A rows at sA[row * CH], W rows at sB[row * CH] (both XOR
// swizzled by row & 7, see the DMA source addresses).
// SKIP: only the wave's first fmv row fragments hold real rows (grouped experts: an expert's
// routed rows end inside the tile) — the others are neither read nor multiplied
template <class C, bool SKIP = false>
__device__ __forceinline__ void mma_tile(const bf16x8* sA, const bf16x8* sB, int lane, int wm, int wn, bool ln_acc,
                                         f32x4 (&acc)[C::FM][C::FN], float (&st_s)[C::FM], float (&st_q)[C::FM],
                                         int fmv = C::FM) {
  // All fragments of the K-tile (both 32-deep halves) are requested before the first MFMA:
  // the second half's ds_reads then complete under the first half's MFMAs instead of
  // behind an lgkmcnt(0) (the compiler counts lgkmcnt per consumer). Wave tiles with more
  // than 12 fragments per half (32 x 224: 2 + 14) load one half at a time — both halves'
  // fragments next to 28 accumulators would not fit the 256 registers of two waves per SIMD.
  constexpr bool HALVES = C::HALF_FRAGS;
  if constexpr (!HALVES) {
    bf16x8 af[2][C::FM], bw[2][C::FN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int row = wn * C::WTN + j * 16 + (lane & 15);
        bw[kk][j] = sB[row * C::CH + (chunk ^ (row & 7))];
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        if (SKIP && i >= fmv) break;
        const int row = wm * C::WTM + i * 16 + (lane & 15);
        af[kk][i] = sA[row * C::CH + (chunk ^ (row & 7))];
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every ds_read ahead of the MFMAs (counted lgkmcnt waits)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (ln_acc) {
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = bf2f(af[kk][i][e]);
            st_s[i] += x;
            st_q[i] += x * x;
          }
      }
      // swapped operands: acc = (W A^T) tile, i.e. C^T — lane holds 4 consecutive output
      // COLUMNS of one row, so the epilogue moves 8-byte vectors instead of bf16 scalars
      if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        if (SKIP && i >= fmv) break;
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16x16x32(bw[kk][j], af[kk][i], acc[i][j]);
      }
      if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(0);
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[C::FM], bw[C::FN];
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int row = wn * C::WTN + j * 16 + (lane & 15);
        bw[j] = sB[row * C::CH + (chunk ^ (row & 7))];
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        if (SKIP && i >= fmv) break;
        const int row = wm * C::WTM + i * 16 + (lane & 15);
        af[i] = sA[row * C::CH + (chunk ^ (row & 7))];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (ln_acc) {
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = bf2f(af[i][e]);
            st_s[i] += x;
            st_q[i] += x * x;
          }
      }
      if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        if (SKIP && i >= fmv) break;
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16x16x32(bw[j], af[i], acc[i][j]);
      }
      if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Joint rings (BXS == 0): A and W rows of a K-tile share one stage and one DMA batch.
// GATHER: A row r is row arows[r] of A (MoE token gather) — a compile-time switch: a runtime
// null check in every launch's prologue cost the GPT-2 GEMMs ~5 %.
// APOL: cache policy of the A rows' DMA (sc1 = 16: A was written in this launch by other
// workgroups' write-through stores — gemm_fused.hip; every other launch keeps 0)
template <class C, bool GATHER = false, int APOL = 0, int WPOL = 0>
__device__ __forceinline__ void mainloop_joint(bf16x8* smem, const bf16* __restrict__ A, int lda,
                                               const bf16* __restrict__ W, int ldw, int M, int N, int m0, int n0,
                                               int kbeg, int nk, int lane, int wave, int kgrp, int wm, int wn,
                                               bool ln_acc, f32x4 (&acc)[C::FM][C::FN], float (&st_s)[C::FM],
                                               float (&st_q)[C::FM], const int* __restrict__ arows) {
  // `wave` is the wave's index in the whole block (all K groups issue DMA); instruction
  // gi = wave*PW + j loads 8 rows of K-tile gi / INSTR of the stage
  const bf16* src[C::PW];
  int dst[C::PW];
#pragma unroll
  for (int j = 0; j < C::PW; ++j) {
    const int gi = C::EVEN ? wave * C::PW + j : min(wave * C::PW + j, C::INSTR * C::KG - 1);  // (repeats: Cfg::PW)
    const int sub = gi / C::INSTR, r8 = gi % C::INSTR;
    const int row = 8 * r8 + (lane >> 3);
    const int gch = (lane & 7) ^ (row & 7);
    const int kofs = kbeg + sub * C::BK + gch * 8;
    if (row < C::BM) {
      int gm = min(m0 + row, M - 1);
      if constexpr (GATHER) gm = arows[gm];  // gathered A rows (MoE: token of each expert-sorted row)
      src[j] = A + (size_t)gm * lda + kofs;
    } else {
      const int gn = min(n0 + row - C::BM, N - 1);
      src[j] = W + (size_t)gn * ldw + kofs;
    }
    dst[j] = sub * C::SUB + r8 * 64;
  }
  bool is_a[C::PW];  // wave-uniform: a DMA instruction covers 8 rows of one operand
#pragma unroll
  for (int j = 0; j < C::PW; ++j) {
    const int gi = C::EVEN ? wave * C::PW + j : min(wave * C::PW + j, C::INSTR * C::KG - 1);
    is_a[j] = 8 * (gi % C::INSTR) < C::BM;
  }
  auto issue = [&](int kt) {
    bf16x8* stage = smem + (kt % C::STAGES) * C::STAGE;
#pragma unroll
    for (int j = 0; j < C::PW; ++j) {
      if constexpr (APOL != 0 || WPOL != 0) {
        if (is_a[j])
          __builtin_amdgcn_global_load_lds((const void*)(src[j] + kt * (C::BK * C::KG)),
                                           (__attribute__((address_space(3))) void*)(stage + dst[j]), 16, 0, APOL);
        else
          __builtin_amdgcn_global_load_lds((const void*)(src[j] + kt * (C::BK * C::KG)),
                                           (__attribute__((address_space(3))) void*)(stage + dst[j]), 16, 0, WPOL);
        continue;
      }
      __builtin_amdgcn_global_load_lds((const void*)(src[j] + kt * (C::BK * C::KG)),
                                       (__attribute__((address_space(3))) void*)(stage + dst[j]), 16, 0, 0);
    }
  };
#pragma unroll
  for (int s = 0; s < C::STAGES - 1; ++s)
    if (s < nk) issue(s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(C::STAGES - 2, nk - 1 - kt);  // tiles issued after kt, still allowed in flight
    wait_tiles<C::PW, C::STAGES - 2>(ahead);
    raw_barrier();
    if (kt + C::STAGES - 1 < nk) issue(kt + C::STAGES - 1);
    const bf16x8* st = smem + (kt % C::STAGES) * C::STAGE + kgrp * C::SUB;
    mma_tile<C>(st, st + C::BM * C::CH, lane, wm, wn, ln_acc, acc, st_s, st_q);
  }
}

// Half-tile ring (256 x 256 tiles, 8 waves as 2 (M) x 4 (N), wave tile 128 x 64).
//
// Why: with whole 64-KiB K-tiles double-buffered (C8) the next tile is issued in one burst
// and waited for with vmcnt(0) one K-tile later; on the GPT-2 LM head every K-tile then
// stalls on the DMA (one 256-tile round of 256x256x768 tiles: 49 us = 2.1 TFLOP/s per CU,
// benchmarks/bench_lmhead.py). Here a K-tile is four 16-KiB HALF-tiles (A rows 0-127,
// A rows 128-255, W rows 0-127, W rows 128-255) in 8 slots (two K-tiles), and the wave's
// 128 x 64 output is computed as four quadrants (64 x 32, 16 MFMAs each) in the order
//   q0 (A top, W left)  q1 (A top, W right)  q2 (A bottom, W right)  q3 (A bottom, W left)
// so a K-tile's W halves are last read in q1 and its A halves in q2: K-tile t+2's W halves
// are issued into them at q2 of K-tile t and its A halves at q3 — four to six quadrant
// phases before they are read, with two to three K-tiles' worth of DMA in flight at all
// times instead of one burst per K-tile.
// Synchronisation (cdna_hip_programming.md §5, "Read a staged buffer one phase AFTER the
// wait that retires it"; RAW / WAR):
//  * q0 of K-tile t: every wave waits (counted vmcnt: only K-tile t+1's 8 DMA instructions
//    may still be outstanding) and then joins the barrier -> t's slots are complete for all;
//  * q2 / q3: a barrier before the DMA issue — every wave has finished (lgkmcnt-waited,
//    consumed by its MFMAs) the reads of the slots being re-filled (W after q1, A after q2).
// Each wave's fragment reads of a quadrant are all issued before its 16 MFMAs.
template <class C, int WPOL = 0>
__device__ __forceinline__ void mainloop_ring(bf16x8* smem, const bf16* __restrict__ A, int lda,
                                              const bf16* __restrict__ W, int ldw, int M, int N, int m0, int n0,
                                              int kbeg, int nk, int lane, int wave, int wm, int wn,
                                              f32x4 (&acc)[C::FM][C::FN]) {
  constexpr int SLOT = 128 * 8;  // bf16x8 units per 16-KiB half-tile slot (128 rows x 128 B)
  // this thread's two DMA pieces of every half-tile: rows 8 * (2 * wave + j) + lane / 8
  const bf16* srcA[2][2];
  const bf16* srcB[2][2];
  int dst[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 8 * (2 * wave + j) + (lane >> 3);
    const int gch = (lane & 7) ^ (r & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      srcA[h][j] = A + (size_t)min(m0 + h * 128 + r, M - 1) * lda + kbeg + gch * 8;
      srcB[h][j] = W + (size_t)min(n0 + h * 128 + r, N - 1) * ldw + kbeg + gch * 8;
    }
    dst[j] = (2 * wave + j) * 64;
  }
  // slot of half-tile kind hk (0 A0, 1 A1, 2 W0, 3 W1) of K-tile t
  auto slot = [&](int t, int hk) { return smem + ((t & 1) * 4 + hk) * SLOT; };
  auto issue = [&](int t, int hk) {
    const bf16* const* src = hk < 2 ? srcA[hk] : srcB[hk - 2];
    bf16x8* st = slot(t, hk);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (hk < 2)  // (hk is a literal at every call: one immediate policy per DMA)
        __builtin_amdgcn_global_load_lds((const void*)(src[j] + t * C::BK),
                                         (__attribute__((address_space(3))) void*)(st + dst[j]), 16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds((const void*)(src[j] + t * C::BK),
                                         (__attribute__((address_space(3))) void*)(st + dst[j]), 16, 0, WPOL);
    }
  };
  // prologue: K-tiles 0 and 1 (W halves first: issue order inside a K-tile does not matter
  // for the counted waits, which retire whole K-tiles)
#pragma unroll
  for (int t = 0; t < 2; ++t)
    if (t < nk) {
      issue(t, 2);
      issue(t, 3);
      issue(t, 0);
      issue(t, 1);
    }
  const int ah = wm;            // the wave's A half (rows 128 * wm ..)
  const int bh = 2 + (wn >> 1);  // its W half
  const int brow0 = (wn & 1) * 64;
  bf16x8 af[2][4], bl[2][2], br[2][2];
  for (int t = 0; t < nk; ++t) {
    // ---- q0: K-tile t complete; A top + W left
    if (t + 1 < nk) wait_vm<8>();
    else wait_vm<0>();
    raw_barrier();
    const bf16x8* sa = slot(t, ah);
    const bf16x8* sb = slot(t, bh);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = i * 16 + (lane & 15);
        af[kk][i] = sa[row * C::CH + (chunk ^ (row & 7))];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = brow0 + j * 16 + (lane & 15);
        bl[kk][j] = sb[row * C::CH + (chunk ^ (row & 7))];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16x16x32(bl[kk][j], af[kk][i], acc[i][j]);
    // ---- q1: A top + W right
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = brow0 + 32 + j * 16 + (lane & 15);
        br[kk][j] = sb[row * C::CH + (chunk ^ (row & 7))];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][2 + j] = mfma16x16x32(br[kk][j], af[kk][i], acc[i][2 + j]);
    // ---- q2: every wave is past its q1 reads -> K-tile t+2's W halves go into t's W slots
    raw_barrier();
    if (t + 2 < nk) {
      issue(t + 2, 2);
      issue(t + 2, 3);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 64 + i * 16 + (lane & 15);
        af[kk][i] = sa[row * C::CH + (chunk ^ (row & 7))];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 + i][2 + j] = mfma16x16x32(br[kk][j], af[kk][i], acc[4 + i][2 + j]);
    // ---- q3: every wave is past its q2 reads -> K-tile t+2's A halves; A bottom + W left
    // (both already in registers)
    raw_barrier();
    if (t + 2 < nk) {
      issue(t + 2, 0);
      issue(t + 2, 1);
    }
    if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 + i][j] = mfma16x16x32(bl[kk][j], af[kk][i], acc[4 + i][j]);
    if constexpr (C::PRIO) __builtin_amdgcn_s_setprio(0);
  }
}

constexpr int kPolStream = 2;  // gfx950 CPol NT (streaming) bit of the DMA's aux operand
constexpr int kPolWT = 16;     // sc1: write-through (the line leaves the XCD's L2 at the store)

// Split rings (BXS > 0): issue order B0 [A0 B1] [A1 B2] ... — iteration t issues
// A(t + SA - 1) then B(t + SB - 1). Waiting for A(t) then leaves a = min(SA-2, nk-1-t)
// later A tiles and b = min(a + 1, nk-1-t) later W tiles in flight (B(t) precedes A(t)).
template <class C, int WPOL = 0, bool SKIP = false, bool GATHER = false>
__device__ __forceinline__ void mainloop_split(bf16x8* smem, const bf16* __restrict__ A, int lda,
                                               const bf16* __restrict__ W, int ldw, int M, int N, int m0, int n0,
                                               int kbeg, int nk, int lane, int wave, int wm, int wn, bool ln_acc,
                                               f32x4 (&acc)[C::FM][C::FN], float (&st_s)[C::FM],
                                               float (&st_q)[C::FM], int fmv, const int* __restrict__ arows) {
  constexpr int D = C::SB - C::SA;  // W tiles issued ahead of the A tile of the same K step
  static_assert(D >= 1, "split rings: the W ring is deeper than the A ring");
  const bf16* srcA[C::PWA];
  const bf16* srcB[C::PWB];
  // SKIP (grouped expert launches, whose row count is the expert's, known on the device only):
  // the A rows come by buffer DMA, and a row past the expert's last one gets an offset past the
  // buffer's end — the load returns zeros WITHOUT a memory request, so the CU's LDS-DMA intake
  // carries only real rows (with clamped addresses every padding row re-read the last one).
  // Every wave still issues the same instructions: the counted vmcnt waits stay exact.
  uint32_t voffA[C::PWA];
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int j = 0; j < C::PWA; ++j) {
    const int row = 8 * (C::EVEN_A ? wave * C::PWA + j : min(wave * C::PWA + j, C::BM / 8 - 1)) + (lane >> 3);
    int gm = min(m0 + row, M - 1);
    if constexpr (GATHER) gm = arows[gm];  // gathered A rows (MoE: token of each expert-sorted row)
    srcA[j] = A + (size_t)gm * lda + kbeg + ((lane & 7) ^ (row & 7)) * 8;
    if constexpr (SKIP)
      voffA[j] = m0 + row < M ? (uint32_t)(((size_t)gm * lda + kbeg + ((lane & 7) ^ (row & 7)) * 8) * 2) : 0x80000000u;
  }
#pragma unroll
  for (int j = 0; j < C::PWB; ++j) {
    const int row = 8 * (C::EVEN_B ? wave * C::PWB + j : min(wave * C::PWB + j, C::BN / 8 - 1)) + (lane >> 3);
    const int gn = min(n0 + row, N - 1);
    srcB[j] = W + (size_t)gn * ldw + kbeg + ((lane & 7) ^ (row & 7)) * 8;
  }
  bf16x8* ringA = smem;
  bf16x8* ringB = smem + C::SA * C::A_STAGE;
  auto issueA = [&](int kt) {
    bf16x8* st = ringA + (kt % C::SA) * C::A_STAGE;
#pragma unroll
    for (int j = 0; j < C::PWA; ++j) {
      auto* dst = (__attribute__((address_space(3))) void*)(st + (C::EVEN_A ? wave * C::PWA + j : min(wave * C::PWA + j, C::BM / 8 - 1)) * 64);
      if constexpr (SKIP)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, voffA[j] + kt * C::BK * 2, 0, 0, 0);
      else
        __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + kt * C::BK), dst, 16, 0, 0);
    }
  };
  auto issueB = [&](int kt) {
    bf16x8* st = ringB + (kt % C::SB) * C::B_STAGE;
#pragma unroll
    for (int j = 0; j < C::PWB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(srcB[j] + kt * C::BK),
                                       (__attribute__((address_space(3))) void*)(st + (C::EVEN_B ? wave * C::PWB + j : min(wave * C::PWB + j, C::BN / 8 - 1)) * 64), 16,
                                       0, WPOL);
  };
  constexpr int DA = C::SA - 1;
#pragma unroll
  for (int q = 0; q < D; ++q)
    if (q < nk) issueB(q);
#pragma unroll
  for (int s = 0; s < DA; ++s) {
    if (s < nk) issueA(s);
    if (s + D < nk) issueB(s + D);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int a = min(DA - 1, nk - 1 - kt);
    // W tiles issued after A(kt): B(kt + D) .. B(min(kt + DA - 1 + D, nk - 1))
    const int b = max(0, min(DA, nk - kt - D));
    if constexpr (D == 1) wait_ab<C::PWA, C::PWB, DA - 1>(a, b);
    else wait_ab_any<C::PWA, C::PWB, DA - 1, DA>(a, b);
    raw_barrier();
    if (kt + DA < nk) issueA(kt + DA);
    if (kt + DA + D < nk) issueB(kt + DA + D);
    mma_tile<C, SKIP>(ringA + (kt % C::SA) * C::A_STAGE, ringB + (kt % C::SB) * C::B_STAGE, lane, wm, wn, ln_acc,
                      acc, st_s, st_q, fmv);
  }
}

// One output tile (tm, tn) over K-slice ks. Everything from here to the end of the epilogue
// is per tile; the kernel below maps blocks to tiles (or loops over a device-side row range).
// LN: row statistics of a folded norm accumulated in the main loop (else, with ln_mode set,
// they come from ep.ext_stats).
// WPOL: cache policy of the split rings' weight DMA (0 default, kPolStream = nt for weights
// read exactly once per step, e.g. MoE experts far larger than the MALL)
// APOL: the A rows' DMA cache policy (joint rings; mainloop_joint); PUB: the output tile is
// stored write-through (sc1) so workgroups of the SAME launch on other XCDs can read it after
// an agent-scope arrival count (gemm_fused.hip) — both 0 / false in every ordinary launch
template <class C, int LN, int WPOL = 0, bool SKIP = false, bool GATHER = false, int APOL = 0, bool PUB = false,
          int SPOL = 0>
__device__ __forceinline__ void glds_tile(bf16x8* smem, const bf16* __restrict__ A, int lda,
                                          const bf16* __restrict__ W, int ldw, bf16* __restrict__ Cp, int ldc,
                                          const bf16* __restrict__ bias, const bf16* __restrict__ R, int ldr,
                                          float* __restrict__ part, int M, int Mmax, int N, int K, int act,
                                          float alpha, int ks, int kslice, int tm, int tn,
                                          const float* __restrict__ ln_colsum, int ln_mode, float ln_eps,
                                          const Epi& ep, const int* __restrict__ arows = nullptr) {
  const RopeArgs& rope = ep.rope;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kgrp = wave / C::NW, wq = wave % C::NW;  // K group, wave within the group
  const int wm = wq / C::WN, wn = wq % C::WN;
  const int m0 = tm * C::BM, n0 = tn * C::BN;
  if (m0 >= M) return;  // whole block idle (uniform: before any barrier)
  DLS_STAMP(0)
  const int kbeg = ks * kslice;
  const int nk = kslice / (C::BK * C::KG);

  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused LayerNorm/RMSNorm prologue: row statistics of A accumulated from the A fragments
  // that stream through LDS anyway (waves with wn == 0; full K per block, splitk == 1)
  const bool ln_acc = LN && ln_mode != 0 && wn == 0;
  float st_s[C::FM], st_q[C::FM];
#pragma unroll
  for (int i = 0; i < C::FM; ++i) st_s[i] = st_q[i] = 0.f;
  if constexpr (C::RING && !SKIP && !GATHER)  // (grouped expert launches keep the joint ring)
    mainloop_ring<C, WPOL>(smem, A, lda, W, ldw, M, N, m0, n0, kbeg, nk, lane, wave, wm, wn, acc);
  else if constexpr (C::BXS > 0)
    mainloop_split<C, WPOL, SKIP, GATHER>(smem, A, lda, W, ldw, M, N, m0, n0, kbeg, nk, lane, wave, wm, wn, ln_acc, acc,
                                  st_s, st_q, min(C::FM, max(0, (M - m0 - wm * C::WTM + 15) / 16)), arows);
  else
    mainloop_joint<C, GATHER, APOL, WPOL>(smem, A, lda, W, ldw, M, N, m0, n0, kbeg, nk, lane, wave, kgrp, wm, wn, ln_acc, acc,
                                    st_s, st_q, arows);
  DLS_STAMP(1)
  if constexpr (C::KG > 1) {
    // sum the K groups' accumulators into group 0 (lane-contiguous 16-B records)
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smem);
    for (int g2 = 1; g2 < C::KG; ++g2) {
      if (kgrp == g2) {
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) red[((i * C::FN + j) * C::NW + wq) * 64 + lane] = acc[i][j];
      }
      __syncthreads();
      if (kgrp == 0) {
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) acc[i][j] += red[((i * C::FN + j) * C::NW + wq) * 64 + lane];
      }
      __syncthreads();
    }
  }

  const int g4 = (lane >> 4) * 4, r16 = lane & 15;
  if (part != nullptr && ep.tile_sem != nullptr) {
    // In-launch split-K combine (cdna_hip_programming.md §projection GEMM item 2, sc1 form):
    // every K slice stores its fp32 tile WRITE-THROUGH (sc1) into its slab, drains, and one
    // lane draws a ticket from the tile's agent-scope counter; the slice that draws
    // splitk-1 reads the other slabs with sc1 loads (no L1 copy can be stale), adds them to
    // its registers and runs the ordinary epilogue. No separate reduce kernel, no spinning.
    const size_t slab = (size_t)Mmax * N;
    const int tiles_m = (M + C::BM - 1) / C::BM;
    int* sem = ep.tile_sem + tm + tn * tiles_m;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(part, 0, (int)(slab * kslice_count(K, kslice) * 4), 0x00020000);
    if (kgrp == 0) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int row = m0 + wm * C::WTM + i * 16 + r16;
        if (row >= M) continue;
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          const int col = n0 + wn * C::WTN + j * 16 + g4;
          if (col >= N) continue;  // N % 8 == 0 on split-K launches: a fragment is in or out whole
          const f32x4 v = acc[i][j];
          u32x4 u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
          __builtin_amdgcn_raw_buffer_store_b128(u, rsrc, (int)(((size_t)ks * slab + (size_t)row * N + col) * 4), 0,
                                                 16);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);  // the block's one LDS array (staging is free now)
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(sem, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == kslice_count(K, kslice) - 1;
      if (last) __hip_atomic_store(sem, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      flag[0] = last;
    }
    __syncthreads();
    const bool last = flag[0] != 0;
    if (!last) return;  // block-uniform
    if (kgrp == 0) {
      const int nsl = kslice_count(K, kslice);
      for (int s2 = 0; s2 < nsl; ++s2) {
        if (s2 == ks) continue;
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
          const int row = min(m0 + wm * C::WTM + i * 16 + r16, M - 1);
#pragma unroll
          for (int j = 0; j < C::FN; ++j) {
            const int col = min(n0 + wn * C::WTN + j * 16 + g4, N - 4);
            const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(
                rsrc, (int)(((size_t)s2 * slab + (size_t)row * N + col) * 4), 0, 16);
            acc[i][j] += f32x4{__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]),
                               __uint_as_float(u[3])};
          }
        }
      }
    }
    part = nullptr;  // the tile now holds the full sum: ordinary epilogue below
  }
  // epilogue: lane (g = lane>>4, r = lane&15) of fragment (i, j) holds C[row][col..col+3]
  // with row = m0 + wm*WTM + 16i + r, col = n0 + wn*WTN + 16j + 4g
  float ln_rs[C::FM], ln_mu[C::FM];
  if (ln_mode != 0) {
    if constexpr (LN) {
    // reduce the 4 lane groups (k-chunks) -> full-row sums, publish per row via LDS
    float* stats = reinterpret_cast<float*>(smem);
    raw_barrier();  // every wave is past its last LDS read of the staging buffers
    if (ln_acc) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        float a = st_s[i], q = st_q[i];
        a += __shfl_xor(a, 16, 64);
        a += __shfl_xor(a, 32, 64);
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        if (lane < 16) {
          const int lr = wm * C::WTM + i * 16 + lane;
          stats[2 * lr] = a;
          stats[2 * lr + 1] = q;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const int lr = wm * C::WTM + i * 16 + r16;
      const float a = stats[2 * lr], q = stats[2 * lr + 1];
      const float inv_k = 1.0f / (float)K;
      if (ln_mode == 1) {
        const float mu = a * inv_k;
        const float var = fmaxf(q * inv_k - mu * mu, 0.f);
        ln_mu[i] = mu;
        ln_rs[i] = rsqrtf(var + ln_eps);
      } else {
        ln_mu[i] = 0.f;
        ln_rs[i] = rsqrtf(q * inv_k + ln_eps);
      }
    }
      } else {
      // statistics handed over by the producer of A (fp32 [M][2] = sum, sum of squares)
      const float inv_k = 1.0f / (float)K;
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int row = min(m0 + wm * C::WTM + i * 16 + r16, M - 1);
        const float a = ep.ext_stats[2 * row], q = ep.ext_stats[2 * row + 1];
        const float mu = ln_mode == 1 ? a * inv_k : 0.f;
        ln_mu[i] = mu;
        ln_rs[i] = rsqrtf(fmaxf(q * inv_k - mu * mu, 0.f) + ln_eps);
      }
    }
  }
  // 8-byte vector stores need 8-B aligned rows (ldc % 4 == 0) — N itself may be ragged
  // (the LM head writes 50257 columns into rows padded to 50304); a fragment whose 4
  // columns straddle N falls back to scalars.
  const bool vec_ok = (ldc % 4 == 0) && (!R || ldr % 4 == 0);
  if (part != nullptr) {  // split-K: fp32 partial slab, reduced by splitk_reduce_kernel
    if (kgrp != 0) return;
    float* P = part + (size_t)ks * Mmax * N;
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const int row = m0 + wm * C::WTM + i * 16 + r16;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int col = n0 + wn * C::WTN + j * 16 + g4;
        if (N % 4 == 0 && col + 3 < N) {
          const f32x4 v = acc[i][j];
          store16_pol<SPOL>(P, ((size_t)row * N + col) * 4,
                            u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                  __float_as_uint(v[3])});
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < N) P[(size_t)row * N + col + e] = acc[i][j][e];
        }
      }
    }
    return;
  }
  if (act == ACT_SWIGLU) {
    if (kgrp != 0) return;
    // fragment pairs (2jj, 2jj+1) hold gate and up for the same 16 output columns
    const int NO = N / 2;
#pragma unroll
    for (int jj = 0; jj < C::FN / 2; ++jj) {
      const int gcol = n0 + wn * C::WTN + jj * 32 + g4;  // gate column in W' space
      const int ocol = (n0 + wn * C::WTN) / 2 + jj * 16 + g4;
      if (ocol >= NO) continue;
      float bg[4] = {0.f, 0.f, 0.f, 0.f}, bu[4] = {0.f, 0.f, 0.f, 0.f};
      float cg[4] = {0.f, 0.f, 0.f, 0.f}, cu[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (bias) {
          bg[e] = bf2f(bias[gcol + e]);
          bu[e] = bf2f(bias[gcol + 16 + e]);
        }
        if (ln_mode != 0) {
          cg[e] = ln_colsum[gcol + e];
          cu[e] = ln_colsum[gcol + 16 + e];
        }
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int row = m0 + wm * C::WTM + i * 16 + r16;
        if (row >= M) continue;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float g = acc[i][2 * jj][e], u = acc[i][2 * jj + 1][e];
          if (ln_mode != 0) {
            g = ln_rs[i] * (g - ln_mu[i] * cg[e]);
            u = ln_rs[i] * (u - ln_mu[i] * cu[e]);
          } else {
            g *= alpha;
            u *= alpha;
          }
          o[e] = f2bf(silu(g + bg[e]) * (u + bu[e]));
        }
        if (vec_ok && ocol + 3 < NO) {
          store8_pol<SPOL>(Cp, ((size_t)row * ldc + ocol) * 2, *reinterpret_cast<const u32x2*>(&o));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ocol + e < NO) Cp[(size_t)row * ldc + ocol + e] = o[e];
        }
      }
    }
    return;
  }
  // Staged epilogue: each wave writes its finished fragments (bias, activation, folded norm,
  // RoPE applied; bf16) into a tile image in LDS, then the block stores the tile as whole
  // 16-B-per-lane row segments (residual add and row statistics on the way out). A lane's
  // fragment holds only 4 columns (8 B) of 16 different rows, so storing fragments directly
  // scatters 32-B pieces over 16 rows per instruction — partial lines that measured
  // ~1.2 TB/s on the 51 MB LM-head output; full rows run at the HBM write rate.
  // BNC 16-B chunks per tile row, stored in rows of BNP (power of two >= 8) chunks: image chunk
  // c of row r sits at c ^ (r & 7), and BNP consecutive lanes own one row in the store pass
  constexpr int BNC = C::BN / 8;
  constexpr int BNP = BNC <= 8 ? 8 : BNC <= 16 ? 16 : BNC <= 32 ? 32 : 64;
  static_assert(C::BN % 8 == 0 && BNC <= 64, "staged epilogue: BN % 8 == 0, BN <= 512");
  static_assert(C::BM * BNP * 16 <= C::LDS_UNITS * 16, "output tile image must fit the staging LDS");
  static_assert((C::BM * BNP) % 64 == 0 && ((C::BM * BNP) % C::T == 0 || C::BM * BNP < C::T),
                "store pass: every wave makes the same number of passes (shuffles stay wave-uniform)");
  bf16* img = reinterpret_cast<bf16*>(smem);
  __syncthreads();  // every wave is done with the staging buffers (and the norm statistics)
  // The activation / folded-norm / RoPE choice is made ONCE per tile and the fragment pass is
  // instantiated per combination: a runtime switch per output value (apply_act) unrolled over
  // the 128 values per lane of a 256 x 256 tile compiled to ~25k instructions of branches
  // around inlined GeLU / SiLU bodies, and the instruction fetches of jumping through them made
  // this pass take 19.5 us per tile on MI355X (benchmarks/gemm_stamps.hip) — 3x the main loop
  // of the GPT-2 LM head.
  auto image_pass = [&](auto act_tag, auto ln_tag, auto rope_tag) {
    constexpr int ACT = decltype(act_tag)::value;
    constexpr bool LNM = decltype(ln_tag)::value, ROPE = decltype(rope_tag)::value;
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      if (kgrp != 0) break;  // K group 0 holds the summed tile
      const int cl = wn * C::WTN + j * 16 + g4;  // local column of this lane's 4 values
      const int col = n0 + cl;
      const bool full = col + 3 < N;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      float csv[4] = {0.f, 0.f, 0.f, 0.f};  // colsum(W') of the 4 columns (folded norm)
      if (bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = col + e < N ? bf2f(bias[col + e]) : 0.f;
      }
      if constexpr (LNM) {
        if (full && (N % 4 == 0)) {
          const f32x4 c4 = *reinterpret_cast<const f32x4*>(ln_colsum + col);
#pragma unroll
          for (int e = 0; e < 4; ++e) csv[e] = c4[e];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) csv[e] = col + e < N ? ln_colsum[col + e] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int rl = wm * C::WTM + i * 16 + r16;
        float v[4];
        if constexpr (LNM) {
          // W.LN(x) = rstd * (W' x - mu * colsum(W')) + (bias + W b), W' = W * ln_w (host-derived)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = act_c<ACT>(ln_rs[i] * (acc[i][j][e] - ln_mu[i] * csv[e]) + bv[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = act_c<ACT>(alpha * acc[i][j][e] + bv[e]);
        }
        if constexpr (ROPE) rope_pairs<4>(v, m0 + rl, col, rope);
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        *reinterpret_cast<bf16x4*>(img + rl * BNP * 8 + (((cl >> 3) ^ (rl & 7)) << 3) + (cl & 7)) = o;
      }
    }
  };
  using B0 = std::integral_constant<bool, false>;
  using B1 = std::integral_constant<bool, true>;
  auto by_ln = [&](auto act_tag, auto rope_tag) {
    if (ln_mode != 0) image_pass(act_tag, B1{}, rope_tag);
    else image_pass(act_tag, B0{}, rope_tag);
  };
  if (rope.cols) {
    by_ln(std::integral_constant<int, ACT_NONE>{}, B1{});  // RoPE epilogues carry no activation
  } else {
    switch (act) {
      case ACT_GELU_TANH: by_ln(std::integral_constant<int, ACT_GELU_TANH>{}, B0{}); break;
      case ACT_SILU: by_ln(std::integral_constant<int, ACT_SILU>{}, B0{}); break;
      case ACT_RELU: by_ln(std::integral_constant<int, ACT_RELU>{}, B0{}); break;
      default: by_ln(std::integral_constant<int, ACT_NONE>{}, B0{}); break;
    }
  }
  __syncthreads();
  DLS_STAMP(2)
  const bool v16 = ((reinterpret_cast<uintptr_t>(Cp) | ((uintptr_t)ldc * 2)) & 15) == 0 &&
                   (!R || ((reinterpret_cast<uintptr_t>(R) | ((uintptr_t)ldr * 2)) & 15) == 0);
  const bf16x8* img8 = reinterpret_cast<const bf16x8*>(img);
  const int tid_ = threadIdx.x;
  // consecutive groups of BNP threads own one tile row per pass (lanes past BNC idle)
#pragma unroll 2
  for (int q = tid_; q < C::BM * BNP; q += C::T) {
    const int rl = q / BNP, cc = q % BNP;
    const int row = m0 + rl, col = n0 + cc * 8;
    bf16x8 o = img8[rl * BNP + (cc ^ (rl & 7))];
    float s1 = 0.f, s2 = 0.f;
    if (cc < BNC && row < M && col < N) {
      if (v16 && col + 8 <= N) {
        if (R) {
          const bf16x8 r8 = *reinterpret_cast<const bf16x8*>(R + (size_t)row * ldr + col);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(o[e]) + bf2f(r8[e]));
        }
        if constexpr (PUB || SPOL != 0) {  // PUB: write-through, the row segment leaves the XCD's
          // L2 for memory; SPOL: the store's cache policy (nt: streaming output)
          const auto rs = __builtin_amdgcn_make_buffer_rsrc(Cp, 0, 0x7fffffff, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(&o), rs,
                                                 (int)(((size_t)row * ldc + col) * 2), 0, PUB ? 16 : SPOL);
        } else {
          *reinterpret_cast<bf16x8*>(Cp + (size_t)row * ldc + col) = o;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float y = bf2f(o[e]);
          s1 += y;
          s2 += y * y;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (col + e >= N) continue;
          float x = bf2f(o[e]);
          if (R) x += bf2f(R[(size_t)row * ldr + col + e]);
          const bf16 ob = f2bf(x);
          Cp[(size_t)row * ldc + col + e] = ob;
          const float y = bf2f(ob);
          s1 += y;
          s2 += y * y;
        }
      }
    }
    if (ep.stats_out) {
#pragma unroll
      for (int o_ = 1; o_ < BNP; o_ <<= 1) {
        s1 += __shfl_xor(s1, o_, 64);
        s2 += __shfl_xor(s2, o_, 64);
      }
      if (cc == 0 && row < M) {
        atomicAdd(ep.stats_out + 2 * row, s1);
        atomicAdd(ep.stats_out + 2 * row + 1, s2);
      }
    }
  }
  DLS_STAMP(3)
}

// LN / RANGED are compile-time switches: a kernel instance carries only the epilogue and
// tile walk it needs (the folded-norm statistics and the row-range loop cost registers).
// POL (plain tiles only): streaming (nt) cache policy of the weight DMA (bit 0, split rings)
// and of the output stores (bit 1) — GemmArgs::stream_pol
// Grouped expert launches: a TALLER tile of the same column width that takes an expert whose
// routed rows overflow C's tile but fit this one in ONE pass over its weight panel (instead of
// a partner block streaming the whole panel again for a few rows). void: none. Specialised
// below the tile configs; enabled by w_stream bit 256 (DLS_EXPERT_TALL).
template <class C>
struct TallTile {
  using type = void;
};
template <class C>
constexpr int tall_lds_units() {
  if constexpr (std::is_void_v<typename TallTile<C>::type>) return 0;
  else return TallTile<C>::type::LDS_UNITS;
}

template <class C, int LN, int RANGED, int POL = 0>
__global__ __launch_bounds__(C::T, C::OCC) void gemm_glds_kernel(const bf16* __restrict__ A, int lda,
                                                         const bf16* __restrict__ W, int ldw, bf16* __restrict__ Cp,
                                                         int ldc, const bf16* __restrict__ bias,
                                                         const bf16* __restrict__ R, int ldr,
                                                         float* __restrict__ part, int M, int N, int K, int act,
                                                         float alpha, int tiles_m, int tiles_n, int splitk,
                                                         int kslice, const float* __restrict__ ln_colsum,
                                                         int ln_mode, float ln_eps, const int* __restrict__ rows,
                                                         int compact_rows, Epi ep) {
  constexpr int kUnits = RANGED == 3 && tall_lds_units<C>() > C::LDS_UNITS ? tall_lds_units<C>() : C::LDS_UNITS;
  __shared__ bf16x8 smem[kUnits];
  const int ntile = tiles_m * tiles_n;
  if constexpr (RANGED == 2) {
    // persistent: a resident grid walks the tiles; tile t+1's first K-tiles are issued right
    // behind tile t's epilogue stores, so the store drain overlaps the next load latency
    // instead of holding the CU (one block per CU cannot overlap them across blocks)
    const int total = ntile * splitk;
    for (int L = blockIdx.x, it = 0; L < total; L += gridDim.x, ++it) {
      if (it) raw_barrier();  // every wave is done reading the previous tile's output image
      const int ks = L / ntile, tile = L % ntile;
      glds_tile<C, LN>(smem, A, lda, W, ldw, Cp, ldc, bias, R, ldr, part, M, M, N, K, act, alpha, ks, kslice,
                       tile % tiles_m, tile / tiles_m, ln_colsum, (LN || ep.ext_stats) ? ln_mode : 0, ln_eps, ep);
    }
    return;
  }
  if constexpr (RANGED == 3) {
    // grouped MoE experts: block (g, tn) walks expert g's row range [rows[g], rows[g+1]) of
    // its column panel with expert g's weight; consecutive blocks share an expert (its rows
    // stay L2-resident while its weight panels stream)
    // (w_stream bit 8: groups sharing weights — panel-major, the panel's groups on one XCD)
    // (w_stream bit 16: row-split PAIRS — blocks b and b + 8 of each 16 sit on the same XCD and
    // start together; the pair splits (g, tn)'s row tiles even / odd, so an expert with more routed
    // rows than one tile streams its weight panel from HBM once, the partner's copy from the L2,
    // instead of a second serial pass re-streaming it: profiles/r6_mixtral/rows_vs_time.txt. The
    // odd partner of an expert that fits one tile exits at once)
    int g = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n, t0 = 0, dt = 1;
    if (ep.w_stream & 8) {
      const int L = xcd_remap(blockIdx.x, gridDim.x), ng = gridDim.x / tiles_n;
      tn = L / ng;
      g = L % ng;
    } else if (ep.w_stream & 16) {
      const int pair = (blockIdx.x >> 4) * 8 + (blockIdx.x & 7);
      if (pair >= tiles_m * tiles_n) return;  // grid rounded up to whole 16-block groups
      g = pair / tiles_n;
      tn = pair % tiles_n;
      t0 = (blockIdx.x >> 3) & 1;
      dt = 2;
    } else if (ep.w_stream & (32 | 64)) {
      // the odd partners as one half of the grid: dispatched after every even block (bit 32) or
      // before them (bit 64). A heavy expert's second row tile then runs on a CU of its own, in
      // parallel with its first, where the serial walk doubled its blocks' time: Mixtral-8x7B
      // 24.74 -> 23.58 ms per step (profiles/r6_ab/expert_pairs.txt)
      const int half = gridDim.x >> 1, second = blockIdx.x >= half, idx = blockIdx.x - second * half;
      t0 = second == ((ep.w_stream & 32) != 0);
      dt = 2;
      g = idx / tiles_n;
      tn = idx % tiles_n;
    }
    if ((ep.w_stream & 128) && !(ep.w_stream & (8 | 16))) {
      // XCD-affine walk (w_stream bit 128): blocks on XCD x (index % 8 under round-robin
      // dispatch) take a CONTIGUOUS run of the (group, column panel) order, so an XCD works
      // through one expert's panels at a time and that expert's rows stay in ITS L2 — the
      // plain order spreads every expert's blocks over all eight XCDs, and each L2 then holds
      // all eight experts' rows (Mixtral down: 8 x 3.7 MB against a 4 MB L2)
      const int total = tiles_m * tiles_n, idx = g * tiles_n + tn;
      const int x = idx & 7, j = idx >> 3, q = total >> 3, r = total & 7;
      const int L = x * q + min(x, r) + j;
      g = L / tiles_n;
      tn = L % tiles_n;
    }
    const int r0 = rows[g], cnt = rows[g + 1] - r0;
    const int Mr = compact_rows ? min(cnt, compact_rows) : cnt;
    const bf16* Wg = reinterpret_cast<const bf16*>(ep.grp_w[g]);
    bf16* Cg = ep.grp_c ? reinterpret_cast<bf16*>(ep.grp_c[g]) : Cp + (size_t)r0 * ldc;
    // gathered A: the group's rows are tokens a_rows[r0 ..]; else rows r0.. of the sorted A.
    // The gather map travels in the `part` argument, unused by grouped launches (no split-K):
    // a new Epi field would change every GEMM launch's argument layout
    const int* a_rows = reinterpret_cast<const int*>(part);
    const int* ag = a_rows ? a_rows + r0 : nullptr;
    const bf16* Ag = a_rows ? A : A + (size_t)r0 * lda;
    if constexpr (!std::is_void_v<typename TallTile<C>::type>) {
      // SPLIT = 2: the taller tile is half as wide — the block and its partner each take one half
      // of the column panel over ALL of the expert's rows (each streams half the panel once; in
      // the serial walk without partners the block takes both halves in turn)
      using T2 = typename TallTile<C>::type;
      constexpr int SPLIT = C::BN / T2::BN;
      static_assert((SPLIT == 1 || SPLIT == 2) && T2::BN * SPLIT == C::BN && T2::BM > C::BM && T2::T == C::T,
                    "a taller tile of the same panel (or of half of it)");
      if ((ep.w_stream & 256) && Mr > C::BM && Mr <= T2::BM) {
        const bool nt = T2::BXS > 0 && (ep.w_stream & 1);
        for (int hh = t0; hh < SPLIT; hh += dt) {  // (SPLIT 1: a partner block has nothing to do)
          if (hh != t0) raw_barrier();
          const int tn2 = tn * SPLIT + hh;
          if (a_rows) {
            if (nt)
              glds_tile<T2, 0, kPolStream, true, true>(smem, Ag, lda, Wg, ldw, Cg, ldc, bias, nullptr, 0, nullptr, Mr,
                                                       M, N, K, act, alpha, 0, K, 0, tn2, ln_colsum, 0, ln_eps, ep, ag);
            else
              glds_tile<T2, 0, 0, false, true>(smem, Ag, lda, Wg, ldw, Cg, ldc, bias, nullptr, 0, nullptr, Mr, M, N,
                                               K, act, alpha, 0, K, 0, tn2, ln_colsum, 0, ln_eps, ep, ag);
          } else {
            if (nt)
              glds_tile<T2, 0, kPolStream, true, false>(smem, Ag, lda, Wg, ldw, Cg, ldc, bias, nullptr, 0, nullptr,
                                                        Mr, M, N, K, act, alpha, 0, K, 0, tn2, ln_colsum, 0, ln_eps, ep,
                                                        ag);
            else
              glds_tile<T2, 0, 0, false, false>(smem, Ag, lda, Wg, ldw, Cg, ldc, bias, nullptr, 0, nullptr, Mr, M, N,
                                                K, act, alpha, 0, K, 0, tn2, ln_colsum, 0, ln_eps, ep, ag);
          }
        }
        return;
      }
    }
#define DLS_GROUPED_WALK(GA)                                                                                      \
  for (int t = t0; t * C::BM < Mr; t += dt) {                                                                      \
    if (t != t0) raw_barrier(); /* every wave is done reading the staging buffers of the previous tile */          \
    if (C::BXS > 0 && (ep.w_stream & 1))                                                                           \
      glds_tile<C, 0, kPolStream, true, GA>(smem, Ag, lda, Wg, ldw, Cg, ldc, bias, nullptr, 0, nullptr, Mr, M, N, K, \
                                            act, alpha, 0, K, t, tn, ln_colsum, 0, ln_eps, ep, ag);                \
    else                                                                                                           \
      glds_tile<C, 0, 0, false, GA>(smem, Ag, lda, Wg, ldw, Cg, ldc, bias, nullptr, 0, nullptr, Mr, M, N, K, act,   \
                                    alpha, 0, K, t, tn, ln_colsum, 0, ln_eps, ep, ag);                             \
  }
    if (a_rows) {
      DLS_GROUPED_WALK(true)
    } else {
      DLS_GROUPED_WALK(false)
    }
#undef DLS_GROUPED_WALK
    return;
  }
  const int bid = xcd_remap(blockIdx.x, ntile * splitk);
  int ks = bid / ntile, tile = bid % ntile;
  int tm = tile % tiles_m, tn = tile / tiles_m;
  if constexpr (!RANGED) {
    if (compact_rows > 0) {
      // XCD-blocked tile order (launch: xcd_block; compact_rows is free on plain launches):
      // XCD x = blockIdx.x % 8 owns an a x b block of output tiles, a = compact_rows M tiles,
      // so its L2 fetches a rows of A panels and b columns of W panels from the MALL instead
      // of all of A (splitk 1, tile counts divisible as the host checked)
      const int a = compact_rows, b = (ntile >> 3) / a, gm = tiles_m / a;
      const int xcd = blockIdx.x & 7, idx = blockIdx.x >> 3;
      tm = (xcd % gm) * a + idx % a;
      tn = (xcd / gm) * b + idx / a;
      ks = 0;
    }
    glds_tile<C, LN, (POL & 1) ? kPolStream : 0, false, false, 0, false,
              ((POL & 2) ? kPolStream : 0) | ((POL & 4) ? kPolWT : 0)>(
        smem, A, lda, W, ldw, Cp, ldc, bias, R, ldr, part, M, M, N, K, act, alpha, ks, kslice, tm, tn, ln_colsum,
        (LN || ep.ext_stats) ? ln_mode : 0, ln_eps, ep);
    return;
  }
  // device-side row range (MoE expert): the host launched ONE tile row (tiles_m == 1) — no
  // idle blocks holding CUs — and each block walks the range's M tiles of its column panel
  const int r0 = rows[0], Mr = compact_rows ? min(rows[1] - r0, compact_rows) : rows[1] - r0;
  A += (size_t)r0 * lda;
  if (!compact_rows) Cp += (size_t)r0 * ldc;
  if (R) R += (size_t)r0 * ldr;
  if (part) part += (size_t)r0 * N;
  for (int t = 0; t * C::BM < Mr; ++t) {
    if (t) raw_barrier();  // every wave is done reading the staging buffers of the previous tile
    glds_tile<C, 0>(smem, A, lda, W, ldw, Cp, ldc, bias, R, ldr, part, Mr, M, N, K, act, alpha, ks, kslice, t, tn,
                    ln_colsum, 0, ln_eps, ep);
  }
}

// XCD-blocked tile order for a plain launch: the M-tile count a of each XCD's a x b block of
// output tiles (a x b = tiles / 8, the 8 blocks tiling the grid) that minimises the operand
// panels one XCD's L2 fetches, a * (A panel bytes) + b * (W panel bytes), when that beats the
// default order (32 consecutive tiles, M fastest) by 10 %; 0 = default order. Off unless
// DLS_XCD_BLOCK=1: on GPT-2's out-proj / fc2 (16 x 16 tiles, 8 x 4 blocks per XCD: 26 % fewer
// panel bytes per L2) the step measured 0.3 % slower (profiles/r4_ab/xcd_grouping.txt).
inline int xcd_block(int tiles_m, int tiles_n, size_t a_bytes, size_t w_bytes) {
  static const bool on = [] {
    const char* e = std::getenv("DLS_XCD_BLOCK");
    return e && *e == '1';
  }();
  const int ntile = tiles_m * tiles_n;
  if (!on || ntile % 8 || ntile < 64) return 0;
  const int per = ntile / 8;
  const size_t cur = (size_t)std::min(per, tiles_m) * a_bytes + (size_t)((per + tiles_m - 1) / tiles_m) * w_bytes;
  size_t best = cur;
  int best_a = 0;
  for (int a = 1; a <= per; ++a) {
    if (per % a || tiles_m % a) continue;
    const int b = per / a;
    if (tiles_n % b || (tiles_m / a) * (tiles_n / b) != 8) continue;
    const size_t c = (size_t)a * a_bytes + (size_t)b * w_bytes;
    if (c < best) {
      best = c;
      best_a = a;
    }
  }
  return best * 10 < cur * 9 ? best_a : 0;
}

// resident blocks of a persistent launch: CUs x blocks per CU (occupancy query, cached)
template <class C, int LN>
int persistent_grid() {
  static int g = 0;
  if (!g) {
    int dev = 0, cus = 256, per = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gemm_glds_kernel<C, LN, 2>, C::T, 0);
    g = cus * (per > 0 ? per : 1);
  }
  return g;
}

template <class C>
bool launch(const GemmArgs& a, int splitk, float* ws, hipStream_t s, const float* ln_colsum, int ln_mode,
            float ln_eps, const int* rows, bool persist) {
  // in-launch combine only while the last arriver's serial read of the other slices stays small
  // (cdna_hip_programming.md: ~1 us per 16 KB; Llama-3-8B's 256x128 split-4 tiles would read
  // 384 KB in one block, far slower than the reduce kernel)
  // (DLS_FIXUP_MAX_KB: the largest slab read, in KiB, for which the combine stays in-launch)
  static const int fixup_max = [] {
    const char* e = std::getenv("DLS_FIXUP_MAX_KB");
    return (e && *e ? std::atoi(e) : 64) * 1024;
  }();
  const bool fixup = splitk > 1 && !rows && (splitk - 1) * C::BM * C::BN * 4 <= fixup_max;
  // policy stores are buffer stores with 32-bit byte offsets from the output's base: outputs
  // (or split-K slabs) of 2 GB and more keep the default stores
  int spol = a.stream_pol & 7;
  if ((size_t)a.M * a.ldc * 2 >= (1ull << 31) || (size_t)a.M * a.N * 4 * splitk >= (1ull << 31)) spol &= 1;
  // ep.w_stream carries the store policy to the split-K reduce kernels (grouped launches alone
  // read it as the weight policy)
  const Epi ep{a.rope, a.stats_out, a.ext_stats, fixup ? a.tile_sem : nullptr, nullptr, nullptr, spol & 4};
  const int crows = rows ? a.compact_rows
                         : (!persist && splitk == 1 ? xcd_block((a.M + C::BM - 1) / C::BM, (a.N + C::BN - 1) / C::BN,
                                                                (size_t)C::BM * a.K * 2, (size_t)C::BN * a.K * 2)
                                                    : 0);
  static_assert(2 * C::BM * sizeof(float) <= C::LDS_UNITS * 16, "LN stats must fit the staging LDS");
  const int tiles_m = rows ? 1 : (a.M + C::BM - 1) / C::BM, tiles_n = (a.N + C::BN - 1) / C::BN;
  const int kslice = a.K / splitk;
  const int total = tiles_m * tiles_n * splitk;
  dim3 grid(total), block(C::T);
#define DLS_K(LN_, RG_, ...)                                                                                      \
  hipLaunchKernelGGL((gemm_glds_kernel<C, LN_, RG_, ##__VA_ARGS__>), grid, block, 0, s, (const bf16*)a.A, a.lda, (const bf16*)a.W, \
                     a.ldw, (bf16*)a.C, a.ldc, (const bf16*)a.bias, (const bf16*)a.R, a.ldr, ws, a.M, a.N, a.K, a.act, \
                     a.alpha, tiles_m, tiles_n, splitk, kslice, ln_colsum, ln_mode, ln_eps, rows, crows, ep)
  const bool ln_in = ln_mode != 0 && !a.ext_stats;
  if (rows) DLS_K(0, 1);
  else if (persist) {
    if (ln_in) {
      if constexpr (C::BM * C::BN <= 256 * 128 && C::KG == 1) {
        grid = dim3(std::min(total, persistent_grid<C, 1>()));
        DLS_K(1, 2);
      }
    } else {
      grid = dim3(std::min(total, persistent_grid<C, 0>()));
      DLS_K(0, 2);
    }
  } else if (ln_in) {
    if constexpr (C::BM * C::BN <= 256 * 128 && C::KG == 1) DLS_K(1, 0);  // 256x256: no registers left for it
  } else {
    const int pol = spol;  // an own kernel per policy
    switch (pol) {
      case 1: DLS_K(0, 0, 1); break;
      case 2: DLS_K(0, 0, 2); break;
      case 3: DLS_K(0, 0, 3); break;
      case 4: DLS_K(0, 0, 4); break;
      case 5: DLS_K(0, 0, 5); break;
      default: DLS_K(0, 0);
    }
  }
#undef DLS_K
  if (splitk > 1 && !ep.tile_sem) return glds_reduce(a, splitk, ws, s, ln_colsum, ln_mode, ln_eps, rows, ep);
  return false;
}

using C0 = Cfg<256, 128, 4, 2, 3>;  // 8 waves, 64x64 per wave: large GEMMs
using C1 = Cfg<128, 128, 2, 2, 3>;  // 4 waves, 64x64 per wave
using C2 = Cfg<128, 64, 2, 2, 4>;   // 4 waves, 64x32 per wave
using C3 = Cfg<64, 64, 2, 2, 4>;    // 4 waves, 32x32 per wave
using C4 = Cfg<64, 128, 2, 2, 4>;
using C5 = Cfg<64, 64, 2, 2, 8>;    // deep pipeline: 7 K-tiles in flight (cold-weight latency)
using C6 = Cfg<128, 64, 2, 2, 6>;   // 5 in flight, 2x rows per block
using C7 = Cfg<128, 128, 2, 2, 4>;
using C8 = Cfg<256, 256, 2, 4, 2>;     // 8 waves, 128x64 per wave, 2 x 64 KiB stages: big square-ish GEMMs
using C9 = Cfg<256, 256, 2, 4, 2, 1>;  // same with s_setprio(1) around the MFMA cluster (T5)
using C10 = Cfg<256, 128, 4, 2, 3, 1>; // C0 with s_setprio
using C11 = Cfg<128, 128, 2, 2, 4, 1>; // C7 with s_setprio
// split rings: the cold weight stream one tile deeper than the L2-resident activations
using C12 = Cfg<256, 256, 2, 4, 2, 0, 1>;  // 2 x 32 KiB A + 3 x 32 KiB W = 160 KiB
using C13 = Cfg<256, 256, 2, 4, 2, 1, 1>;
using C14 = Cfg<256, 128, 4, 2, 3, 0, 1>;  // 3 x 32 KiB A + 4 x 16 KiB W = 160 KiB
using C15 = Cfg<128, 128, 2, 2, 3, 0, 1>;  // 3 x 16 KiB A + 4 x 16 KiB W
// two K groups (8 waves, intra-block split-K) for the skinny M = 512 GEMMs
using C16 = Cfg<64, 64, 2, 2, 3, 0, 0, 2>;   // 3 x 32 KiB stages
using C17 = Cfg<64, 64, 2, 2, 2, 0, 0, 2>;   // 2 x 32 KiB: two blocks per CU
using C18 = Cfg<128, 64, 2, 2, 2, 0, 0, 2>;  // 2 x 48 KiB
using C19 = Cfg<64, 128, 2, 2, 2, 0, 0, 2>;
using C20 = Cfg<64, 64, 2, 2, 2, 0, 0, 4>;   // four K groups: 16 waves, 2 x 64 KiB stages
using C21 = Cfg<64, 64, 1, 2, 2, 0, 0, 4>;   // four K groups of 2 waves (64x32 each)
// tiles sized so a 512-row GEMM covers the 256 CUs exactly once (per-CU L2->LDS bytes, not
// MFMA rate, bound these: 512x3072 -> 8x32 tiles of 64x96, 512x2304 -> 16x16 of 32x144,
// 512x768 -> 16x16 of 32x48)
using C22 = Cfg<64, 96, 2, 2, 4>;
using C23 = Cfg<32, 144, 2, 1, 4>;
using C24 = Cfg<32, 48, 2, 1, 4>;
using C25 = Cfg<64, 96, 2, 2, 3, 0, 0, 2>;
using C26 = Cfg<32, 144, 2, 1, 3, 0, 0, 2>;
using C27 = Cfg<32, 48, 2, 1, 4, 0, 0, 2>;
// 128x128 with two K groups: each stage's DMA covers 256 contiguous bytes of every weight row
// (two K-tiles back to back) — the HBM-streaming MoE expert GEMMs (128 routed rows, cold weights)
using C28 = Cfg<128, 128, 2, 2, 2, 0, 0, 2>;
// 192-row tiles: a top-2 expert of a 512-token batch gets ~128 +- 11 routed rows, so 128-row
// tiles need a second pass over the WHOLE weight panel for most experts; 192 rows take any
// such expert in one pass (its weights stream from HBM exactly once)
using C29 = Cfg<192, 128, 2, 2, 3>;
using C30 = Cfg<192, 128, 2, 2, 2, 0, 0, 2>;
using C31 = Cfg<192, 128, 2, 2, 2, 0, 1>;  // split rings: 2 x 24 KiB A + 3 x 16 KiB W
// deeper split rings for the HBM-streaming expert GEMMs: 3 x 24 KiB A + 4 x 16 KiB W = 136 KiB
// keeps 2 A and 3 W tiles in flight (C31: 1 and 2); C33 issues them from 8 waves (48 x 64 wave
// tiles). Measured (Mixtral-8x7B grouped launches): C33 441 / 206 us for gate-up / down vs C31
// 465 / 215; C32 (same rings, 4 waves) no faster than C31 — the wave count, not the ring
// depth, moved it. A 192 x 256 tile (half the routed-row bytes per weight byte) ran > 550 us.
// Role-split rings (half the waves DMA only W, 5-6 tiles deep; the other half only A, 2 deep;
// 8 or 16 waves) were slower still: 537-545 / 254-268 us — not bytes in flight but the number of
// DMA-issuing waves per stream bounds these launches.
using C32 = Cfg<192, 128, 2, 2, 3, 0, 1>;
using C33 = Cfg<192, 128, 4, 2, 3, 0, 1>;
// 256 x 256 with the half-tile ring main loop (mainloop_ring): LM heads and the large GEMMs
using C34 = Cfg<256, 256, 2, 4, 2, 0, 0, 1, 1>;
using C35 = Cfg<256, 256, 2, 4, 2, 1, 0, 1, 1>;
// 224-column tiles: a 512-row GEMM whose N is a multiple of 7 x 32 fills the 256 CUs in whole
// rounds (Llama-3-8B gate/up N = 28672 -> 2 x 128 = 256 tiles of 256 x 224; 256 x 256 leaves 32
// CUs idle), and the GPT-2 LM head (N = 50304) takes 450 tiles = 1.76 rounds instead of 394
// tiles of 256 x 256 whose second round is half empty. Split rings: 2 x 32 KiB A + 3 x 28 KiB W.
using C36 = Cfg<256, 224, 4, 2, 2, 0, 1>;  // wave 64 x 112 (plain epilogues)
using C37 = Cfg<256, 224, 8, 1, 2, 0, 1>;  // wave 32 x 224: SwiGLU gate/up pairs (multiples of 32)
// 128 x 96 / 128 x 64 tiles of 8 waves for the long-K projections (K = 4096: 512 x 6144 ->
// 4 x 64 = 256 tiles, 512 x 4096 -> 4 x 64 = 256 tiles of 128 x 64) without split-K partials
using C38 = Cfg<128, 96, 4, 2, 4>;             // wave 32 x 48, 4 x 28 KiB stages
using C39 = Cfg<128, 96, 2, 2, 2, 0, 0, 2>;    // two K groups of wave 64 x 48, 2 x 56 KiB stages
using C40 = Cfg<128, 64, 2, 2, 3, 0, 0, 2>;    // two K groups of wave 64 x 32, 3 x 48 KiB stages
// MoE experts (192 routed rows, cold weights): the W ring TWO tiles deeper than the A ring —
// 3 x 24 KiB A + 5 x 16 KiB W = 152 KiB, four weight tiles (64 KiB) in flight per CU (C33: 3)
using C41 = Cfg<192, 128, 4, 2, 3, 0, 2>;
// 256 x 144 tiles of 8 waves (wave 32 x 144): the TAIL of a wide GEMM whose first columns ran
// as one whole round of 256 x 256 tiles — the GPT-2 LM head's last 17,489 columns as 244 tiles
// (one round) instead of 138 more 256 x 256 tiles that leave 118 CUs idle (ops.linear_norm
// column split, ops/gemm_tuning.json "col_splits"). 3 x 50 KiB joint stages.
using C42 = Cfg<256, 144, 8, 1, 3>;
// 256 x 192 tiles, 8 waves as 4 x 2 (wave 64 x 96), split rings 2 x 32 KiB A + 3 x 24 KiB W:
// with split-K 4 a 512 x 6144 x 4096 projection (Llama-3 QKV) is 64 tiles x 4 slices = 256
// blocks whose per-CU operand bytes are half those of the one-slice 128 x 96 tiles
using C43 = Cfg<256, 192, 4, 2, 2, 0, 1>;
// MoE gate/up: 160 routed rows (an expert's whole row range at 512 tokens top-2 over 8 experts)
// x 256 weight columns, wave 80 x 64, split rings 2 x 20 KiB A + 3 x 32 KiB W: 80 B of operand
// intake per output instead of 102 for 192 x 128 (the gathered A rows are re-read per column tile)
using C44 = Cfg<160, 256, 2, 4, 2, 0, 1>;
// GPT-2's skinny N = 768 GEMMs: 32 x 48 tiles with FOUR K groups (8 waves issuing the LDS-DMA
// of each 256-deep super-step instead of 4): more DMA issuers per CU for the intake-bound K loop
using C45 = Cfg<32, 48, 2, 1, 3, 0, 0, 4>;
// Two workgroups per CU (the MoE expert launches expose per-workgroup latency
// with one 512-thread workgroup per CU): 4-wave 128 x 128 tiles in at most 80 KiB of LDS, so a
// second workgroup's DMA and MFMAs run while the first waits at its barrier — joint rings of 2
// stages (64 KiB), and split rings with the weight ring one deeper (2 x 16 KiB A + 3 x 16 KiB W)
using C46 = Cfg<128, 128, 2, 2, 2, 0, 0, 1, 0, 2>;
using C47 = Cfg<128, 128, 2, 2, 2, 0, 1, 1, 0, 2>;
// (measured and dropped: the same tile with 2 or 4 stages, with eight K groups, and fc1 as one
// round of 64 x 96 tiles with four K groups — profiles/r4_ab/gpt2_n768_cfg45.txt)
// (and the MoE experts' 192 x 128 tile with two K groups, 16 waves: Mixtral 28.7 / 42.6 ms
// with it on down / gate-up against 24.3 — profiles/r4_ab/moe_gateup_cfg44.txt)

// the Mixtral down tile's taller form (busiest expert per layer: 149-227 routed rows,
// profiles/r6_mixtral/rows_vs_time.txt): 192 -> 256 rows (config 14; the grouped kernel keeps
// 241 VGPRs, no scratch). The gate/up tile's (160 -> 224 rows, wave 112 x 64) spilled 68 VGPRs
// in the grouped kernel: not instantiated.
// gate/up (160 x 256): 224 x 256 (wave 112 x 64, split rings 2 x 28 KiB A + 3 x 32 KiB W) — the
// grouped kernel spills 68 VGPRs with it (a 320 x 128 half-panel form spilled 132-172)
template <>
struct TallTile<C44> {
  using type = Cfg<224, 256, 2, 4, 2, 0, 1>;
};
template <>
struct TallTile<C33> {
  using type = C14;
};

template <class C>
void grouped(const GemmArgs& a, int n_groups, const int* offsets, const unsigned long long* w_ptrs,
             const unsigned long long* c_ptrs, hipStream_t s, const int* a_rows) {
  // expert weights (read once per step, far larger than the MALL) are DMA'd with the nt
  // policy: Mixtral-8x7B 27.05 vs 27.89 ms per step (DLS_EXPERT_NT=0 restores the default)
  static const int w_stream = [] {
    const char* e = std::getenv("DLS_EXPERT_NT");
    return e && e[0] == '0' ? 0 : 1;
  }();
  // (the nt path DMAs the A rows by buffer loads with 32-bit offsets: an A of 2 GB or more
  // takes the default path)
  // row-split pairs (kernel: RANGED == 3): DLS_EXPERT_PAIRS=0 one block walks every row tile,
  // 1 same-XCD partners, 2 (default) partners in the grid's second half, 3 in its first half
  // (read per launch — a captured step replays without it — so a test can switch modes)
  const char* pe = std::getenv("DLS_EXPERT_PAIRS");
  const int pairs = pe && *pe ? std::atoi(pe) : 2;
  const int pair = a.grouped_shared ? 0 : pairs;
  // DLS_EXPERT_XCD=1: XCD-affine block order (kernel: RANGED == 3)
  const char* xe = std::getenv("DLS_EXPERT_XCD");
  const bool xcd = xe && *xe == '1' && !a.grouped_shared && pair != 1;
  // DLS_EXPERT_TALL (default 1): an expert past the tile's rows but within its TallTile's takes
  // one taller pass (configs with a TallTile only): Mixtral-8x7B 24.18-24.25 -> 23.72-23.81 ms
  // (profiles/r6_ab/expert_tall_tile.txt)
  const char* te = std::getenv("DLS_EXPERT_TALL");
  const bool tall = !(te && *te == '0') && !a.grouped_shared;
  const Epi ep{a.rope, nullptr, nullptr, nullptr, w_ptrs, c_ptrs,
               (a.grouped_shared ? 8 : ((size_t)a.M * a.lda * 2 < (1ull << 31) ? w_stream : 0)) |
                   (pair == 1 ? 16 : pair == 2 ? 32 : pair == 3 ? 64 : 0) | (xcd ? 128 : 0) | (tall ? 256 : 0)};
  const int tiles_n = (a.N + C::BN - 1) / C::BN;
  const int blocks = pair == 1 ? (n_groups * tiles_n + 7) / 8 * 16 : pair >= 2 ? 2 * n_groups * tiles_n
                                                                               : n_groups * tiles_n;
  // (tiles_m carries the group count: the paired walk bounds its pair index by it)
  hipLaunchKernelGGL((gemm_glds_kernel<C, 0, 3>), dim3(blocks), dim3(C::T), 0, s, (const bf16*)a.A, a.lda,
                     nullptr, a.ldw, (bf16*)a.C, a.ldc, nullptr, nullptr, 0,
                     const_cast<float*>(reinterpret_cast<const float*>(a_rows)), a.M, a.N, a.K, a.act, a.alpha,
                     n_groups, tiles_n, 1, a.K, nullptr, 0, 1e-5f, offsets, a.compact_rows, ep);
}

}  // namespace

// external entry points of config ID (declared in gemm_glds_cfgs.h)
#define DLS_GLDS_DEFINE(ID)                                                                                     \
  bool glds_launch_cfg##ID(const GemmArgs& a, int splitk, float* ws, hipStream_t s, const float* ln_colsum,     \
                           int ln_mode, float ln_eps, const int* rows, bool persist) {                          \
    return launch<C##ID>(a, splitk, ws, s, ln_colsum, ln_mode, ln_eps, rows, persist);                          \
  }                                                                                                             \
  void glds_grouped_cfg##ID(const GemmArgs& a, int n_groups, const int* offsets, const unsigned long long* w_ptrs, \
                            const unsigned long long* c_ptrs, hipStream_t s, const int* a_rows) {               \
    grouped<C##ID>(a, n_groups, offsets, w_ptrs, c_ptrs, s, a_rows);                                            \
  }
