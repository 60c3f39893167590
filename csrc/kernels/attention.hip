// Flash-style attention forward on MFMA (causal or full, MHA or GQA), bf16 in/out.
//
// One workgroup = 64 query rows of one (batch, head): 4 waves x 16 rows. Per 64-key
// tile: K is staged row-major into LDS (16-B chunks XOR-swizzled by row, T2) and V is
// staged transposed (V^T[d][key]) so both MFMA products read their B fragments as
// contiguous 16-byte LDS vectors:
//   S  = Q K^T   mfma_f32_16x16x32_bf16, Q fragments held in registers for the whole loop
//   O += P V     P goes through a per-wave LDS tile to move from the accumulator layout
//                (row = 4*(l>>4)+i) to the A-operand layout (row = l&15)
// Online softmax keeps (m, l) per row in fp32 with exp2 and a log2(e)-prescaled scale;
// rows reduce across the 16 lanes of an MFMA column group with 4 xor-shuffles.
// The score matrix never touches HBM. Causal blocks stop at their diagonal tile.
#include "common.h"
#include "kernels.h"

namespace {

template <int D>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16* __restrict__ Q, int ldq,
                                                       const bf16* __restrict__ Kp, int ldk,
                                                       const bf16* __restrict__ Vp, int ldv, bf16* __restrict__ O,
                                                       int ldo, int S, int n_head, int n_kv_head, float scale_log2,
                                                       int causal) {
  constexpr int KT = 64;            // keys per tile
  constexpr int CH = D / 8;         // 16-B chunks per K row
  constexpr int VCH = KT / 8;       // 16-B chunks per V^T row
  constexpr int ND = D / 16;        // output fragments per wave
  constexpr int NQK = D / 32;       // k-steps of Q K^T
  __shared__ bf16x8 smem[KT * CH + D * VCH + 4 * 16 * VCH];
  bf16x8* Ks = smem;
  bf16x8* Vt = smem + KT * CH;
  bf16x8* Ps = Vt + D * VCH;
  bf16* Vt_e = reinterpret_cast<bf16*>(Vt);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int g = h / (n_head / n_kv_head);
  const int q0 = qt * 64;
  const size_t tok0 = (size_t)b * S;

  // Q fragments for this wave's 16 rows (A operand: row l&15, k = 8*(l>>4)+j)
  bf16x8 qf[NQK];
  {
    const int row = q0 + wave * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < NQK; ++kk) {
      const int d = kk * 32 + 8 * (lane >> 4);
      qf[kk] = row < S ? *reinterpret_cast<const bf16x8*>(Q + (tok0 + row) * ldq + h * D + d) : bf16x8{};
    }
  }
  f32x4 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_i[4], l_i[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m_i[i] = -INFINITY;
    l_i[i] = 0.f;
  }

  const int kv_end = causal ? min(S, q0 + 64) : S;
  for (int k0 = 0; k0 < kv_end; k0 += KT) {
    __syncthreads();  // previous tile fully consumed
    // stage K (row-major, swizzled) and V^T
#pragma unroll
    for (int it = 0; it < (KT * CH) / 256; ++it) {
      const int qd = tid + it * 256, row = qd / CH, c = qd % CH;
      const int key = k0 + row;
      bf16x8 kv = {}, vv = {};
      if (key < S) {
        kv = *reinterpret_cast<const bf16x8*>(Kp + (tok0 + key) * ldk + g * D + c * 8);
        vv = *reinterpret_cast<const bf16x8*>(Vp + (tok0 + key) * ldv + g * D + c * 8);
      }
      Ks[row * CH + (c ^ (row & (CH - 1)))] = kv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = c * 8 + e;
        Vt_e[(d * VCH + ((row >> 3) ^ (d & 7))) * 8 + (row & 7)] = vv[e];
      }
    }
    __syncthreads();

    // S = Q K^T : 16 rows x 64 keys per wave
    f32x4 s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = n * 16 + (lane & 15);
#pragma unroll
      for (int kk = 0; kk < NQK; ++kk) {
        const int chunk = kk * 4 + (lane >> 4);
        s[n] = mfma16x16x32(qf[kk], Ks[row * CH + (chunk ^ (row & (CH - 1)))], s[n]);
      }
    }
    // mask + online softmax (rows 4*(l>>4)+i, keys n*16 + (l&15))
    const int qrow_base = q0 + wave * 16 + 4 * (lane >> 4);
    float p[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qrow = qrow_base + i;
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int key = k0 + n * 16 + (lane & 15);
        float v = s[n][i] * scale_log2;
        if (key >= S || (causal && key > qrow)) v = -INFINITY;
        p[n][i] = v;
        mx = fmaxf(mx, v);
      }
      mx = group16_max(mx);
      const float m_new = fmaxf(m_i[i], mx);
      const float alpha = (m_new == -INFINITY) ? 1.f : exp2f(m_i[i] - m_new);
      float sum = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float e = (m_new == -INFINITY) ? 0.f : exp2f(p[n][i] - m_new);
        p[n][i] = e;
        sum += e;
      }
      sum = group16_sum(sum);
      l_i[i] = l_i[i] * alpha + sum;
      m_i[i] = m_new;
#pragma unroll
      for (int dn = 0; dn < ND; ++dn) o[dn][i] *= alpha;
    }
    // P -> per-wave LDS tile [16 rows][64 keys], swizzled by row
    bf16* Pw = reinterpret_cast<bf16*>(Ps + wave * 16 * VCH);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * (lane >> 4) + i;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = n * 16 + (lane & 15);
        Pw[(r * VCH + ((col >> 3) ^ (r & 7))) * 8 + (col & 7)] = f2bf(p[n][i]);
      }
    }
    __syncthreads();
    // O += P V
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r = lane & 15, chunk = kk * 4 + (lane >> 4);
      const bf16x8 pf = Ps[wave * 16 * VCH + r * VCH + (chunk ^ (r & 7))];
#pragma unroll
      for (int dn = 0; dn < ND; ++dn) {
        const int d = dn * 16 + (lane & 15);
        o[dn] = mfma16x16x32(pf, Vt[d * VCH + (chunk ^ (d & 7))], o[dn]);
      }
    }
  }
  // normalise and store
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qrow = q0 + wave * 16 + 4 * (lane >> 4) + i;
    if (qrow >= S) continue;
    const float inv = l_i[i] > 0.f ? 1.f / l_i[i] : 0.f;
    bf16* orow = O + (tok0 + qrow) * ldo + h * D;
#pragma unroll
    for (int dn = 0; dn < ND; ++dn) orow[dn * 16 + (lane & 15)] = f2bf(o[dn][i] * inv);
  }
}

}  // namespace

void launch_attention_fwd(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.S + 63) / 64, a.n_head, a.B), block(256);
  const float sl2 = a.scale * 1.4426950408889634f;
  const bf16* q = static_cast<const bf16*>(a.q);
  const bf16* k = static_cast<const bf16*>(a.k);
  const bf16* v = static_cast<const bf16*>(a.v);
  bf16* o = static_cast<bf16*>(a.o);
  if (a.D == 64)
    hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, block, 0, s, q, a.ldq, k, a.ldk, v, a.ldv, o, a.ldo, a.S,
                       a.n_head, a.n_kv_head, sl2, a.causal);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, block, 0, s, q, a.ldq, k, a.ldk, v, a.ldv, o, a.ldo, a.S,
                       a.n_head, a.n_kv_head, sl2, a.causal);
}
