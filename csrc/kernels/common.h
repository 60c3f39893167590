// Shared CDNA4 (gfx950) helpers for the hand-written kernels.
//
// Conventions used by every kernel in this directory:
//  * wave64: lane = threadIdx.x & 63, wave = threadIdx.x >> 6; block sizes are
//    multiples of 64.
//  * bf16 storage as clang's native __bf16; math in fp32. Conversions use plain casts,
//    which hipcc lowers to v_cvt_pk_bf16_f32 (NaN-preserving, RNE).
//  * global memory is touched in 16-byte vectors (8 x bf16) wherever the layout allows
//    (cdna_hip_programming.md Guideline 13: scalar bf16 loads cost 2-2.5x).
//  * MFMA: __builtin_amdgcn_mfma_f32_16x16x32_bf16. Operand maps (lane l):
//      A[row l&15][k 8*(l>>4)+j], B[k 8*(l>>4)+j][col l&15], j = 0..7
//      C/D[row 4*(l>>4)+i][col l&15], i = 0..3
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Vector stores with an explicit cache policy (aux bits: 2 nt, 16 sc1 = write-through) at a
// per-lane byte offset from a workgroup-uniform base (the buffer resource lives in SGPRs).
// Write-through leaves no dirty line of the output in the XCD's L2 for the kernel boundary to
// write back. POL 0: a plain store.
template <int POL>
__device__ __forceinline__ void store16_pol(void* base, size_t off, u32x4 v) {
  if constexpr (POL == 0) {
    *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(base) + off) = v;
  } else {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)off, 0, POL);
  }
}
template <int POL>
__device__ __forceinline__ void store8_pol(void* base, size_t off, u32x2 v) {
  if constexpr (POL == 0) {
    *reinterpret_cast<u32x2*>(reinterpret_cast<char*>(base) + off) = v;
  } else {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(v, rs, (int)off, 0, POL);
  }
}

#define DLS_WAVE 64

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reductions inside aligned groups of 16 lanes (one MFMA 16x16 column group)
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float gelu_tanh(float x) {
  // 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))) == x * sigmoid(2u)
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return x / (1.0f + __expf(-2.0f * u));
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD (blocks b, b+8, ... share one), so
// neighbouring output tiles that share operand panels hit the same private L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg <= 8) return orig;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8, idx = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// ACT_SWIGLU: GEMM epilogue silu(gate) * up over a weight whose rows interleave gate and up
// in blocks of 16 (W' rows 32c..32c+15 = gate 16c.., 32c+16..32c+31 = up 16c..); output N/2 wide
enum DlsAct : int { ACT_NONE = 0, ACT_GELU_TANH = 1, ACT_SILU = 2, ACT_RELU = 3, ACT_SWIGLU = 4 };

// compile-time activation (epilogues instantiated per activation: no per-value branch)
template <int ACT>
__device__ __forceinline__ float act_c(float v) {
  if constexpr (ACT == ACT_GELU_TANH) return gelu_tanh(v);
  else if constexpr (ACT == ACT_SILU) return silu(v);
  else if constexpr (ACT == ACT_RELU) return fmaxf(v, 0.f);
  else return v;
}

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case ACT_GELU_TANH: return gelu_tanh(v);
    case ACT_SILU: return silu(v);
    case ACT_RELU: return fmaxf(v, 0.f);
    default: return v;
  }
}

// rotate the adjacent column pairs (c, c+1) of v[0..n) that start at output column col
// (even) of row `row` — see RopeArgs
template <int NV>
__device__ __forceinline__ void rope_pairs(float* v, int row, int col, const RopeArgs& rp) {
  if (col >= rp.cols) return;
  const int half = rp.D >> 1;
  const int pos = row % rp.S;
  const int j0 = (col % rp.D) >> 1;
  const float* cp = rp.cos + (size_t)pos * half + j0;
  const float* sp = rp.sin + (size_t)pos * half + j0;
#pragma unroll
  for (int p = 0; p < NV / 2; ++p) {
    const float c = cp[p], sn = sp[p];
    const float x0 = v[2 * p], x1 = v[2 * p + 1];
    v[2 * p] = x0 * c - x1 * sn;
    v[2 * p + 1] = x1 * c + x0 * sn;
  }
}
