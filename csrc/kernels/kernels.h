// Host-side launchers for the HIP/CDNA4 kernels (raw pointers + hipStream_t, so the
// torch binding translation unit does not need the device compiler's headers).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

constexpr int kActSwiglu = 4;  // == ACT_SWIGLU in common.h (device-side enum)

// RoPE applied in a GEMM epilogue to output columns [0, cols): the q/k rows of the weight are
// PAIR-INTERLEAVED per head (column 2i <-> d_i, 2i+1 <-> d_{i+D/2}), so a rotary pair is two
// adjacent columns of one lane; position = row % S; cos/sin tables are fp32 [S][D/2].
struct RopeArgs {
  const float* cos = nullptr;
  const float* sin = nullptr;
  int S = 1, D = 2, cols = 0;  // cols == 0: off
};

struct GemmArgs {
  const void* A;  // bf16 [M][lda]
  int lda;
  const void* W;  // bf16 [N][ldw]
  int ldw;
  void* C;        // bf16 [M][ldc]
  int ldc;
  const void* bias;  // bf16 [N] or nullptr
  const void* R;     // bf16 [M][ldr] residual or nullptr
  int ldr;
  int M, N, K;
  int act;       // DlsAct
  float alpha;
  int config;    // -1 = auto
  int compact_rows = 0;  // > 0 with a device row range [r0, r1): write output rows 0..r1-r0-1 (not r0..),
                         // and at most compact_rows of them (the output's row capacity)
  // grouped launches whose groups share weights (a cross-request expert batch: one group per
  // (request, expert)): the groups of one weight panel run on consecutive workgroups of one XCD
  // and the weights keep the default cache policy, so each panel comes from HBM once
  int grouped_shared = 0;
  RopeArgs rope{};
  // Row statistics hand-off between a residual-producing GEMM and the next folded norm:
  // stats_out: fp32 [M][2] (zeroed by the caller) += (sum, sum of squares) of each FINAL
  //            (bf16-rounded) output row — the producer's epilogue emits them for free;
  // ext_stats: read them instead of accumulating them in the consumer's main loop (with
  //            ln_mode 1/2 and ln_colsum: any tile config, split-K allowed).
  float* stats_out = nullptr;
  const float* ext_stats = nullptr;
  int* tile_sem = nullptr;  // split-K: >= tiles_m*tiles_n zeroed counters -> combine inside the GEMM launch
  // post-norm of the FINAL output rows for the next (unfolded) norm: norm_out[M][ldn] =
  // norm(C) * norm_w (+ norm_b); norm_mode 1 LayerNorm, 2 RMSNorm. Split-K launches do it in
  // their row-owning reduce (no separate norm launch); launch_gemm_glds reports whether it did.
  void* norm_out = nullptr;
  const void* norm_w = nullptr;
  const void* norm_b = nullptr;
  int norm_mode = 0;
  float norm_eps = 1e-5f;
  int ldn = 0;
  // cache policy of a plain split-ring launch (LN 0): bit 0 the weight DMA streams (nt), bit 1
  // the output stores stream (nt) — for a weight read once per step and a write-once output
  // (the LM head's 77 MB weight and 51 MB of logits) that should not displace the layer
  // weights from the Infinity Cache
  int stream_pol = 0;
};

// epilogue extras carried down to the tile code
struct Epi {
  RopeArgs rope;
  float* stats_out;
  const float* ext_stats;
  // in-launch split-K combine: one arrival counter per output tile (zero before the launch,
  // reset by each tile's last arriver); nullptr -> separate reduce kernel
  int* tile_sem = nullptr;
  // grouped launch (every expert of an MoE layer in ONE grid): per-group weight pointers and,
  // for compact outputs, per-group output pointers (device arrays of E addresses)
  const unsigned long long* grp_w = nullptr;
  const unsigned long long* grp_c = nullptr;
  // grouped launch: weight DMA with the streaming (nt) cache policy (split-ring configs)
  int w_stream = 0;
};

int gemm_pick_config(int M, int N, int K);
void launch_gemm_bf16(const GemmArgs& a, hipStream_t s);  // register-staged, any K % 8 == 0

// LDS-DMA multistage GEMM (K % 64 == 0); split-K partials need workspace_bytes of fp32
int gemm_glds_num_configs();
int gemm_glds_kstep(int cfg);  // K granularity of a config (64, or 128 for two K groups)
// cfg | kGemmPersist: the same tile config as a persistent launch (a resident grid walks the
// tiles; one tile's store drain overlaps the next tile's first loads)
constexpr int kGemmPersist = 64;
void gemm_glds_pick(int M, int N, int K, int* cfg, int* splitk);
size_t gemm_glds_workspace_bytes(int M, int N, int splitk);
// ln_mode: 0 none, 1 LayerNorm, 2 RMSNorm folded into the GEMM (A = raw input rows,
// W pre-scaled by the norm gain, ln_colsum[n] = sum_k W[n][k], bias = bias + W.ln_bias)
// rows (device int32[2], optional): only rows [rows[0], rows[1]) of A/C/R take part (M is then
// the maximum row count, sizing the grid) — an MoE expert's routed rows without a host sync.
// returns true when the launch also wrote a.norm_out (a split-K GEMM's row-owning reduce)
bool launch_gemm_glds(const GemmArgs& a, int cfg, int splitk, void* workspace, hipStream_t s,
                      const float* ln_colsum = nullptr, int ln_mode = 0, float ln_eps = 1e-5f,
                      const int* rows = nullptr);
// Grouped MoE-expert GEMM: E groups in ONE launch (grid = E x column tiles). Group g multiplies
// rows [offsets[g], offsets[g+1]) of A by its own weight (w_ptrs[g], [N][K], ldw = a.ldw) and
// writes them either at the same rows of a.C (c_ptrs == nullptr) or compactly to rows
// 0..min(count, a.compact_rows)-1 of c_ptrs[g]. No split-K; any LDS-DMA config.
void launch_gemm_glds_grouped(const GemmArgs& a, int cfg, int n_groups, const int* offsets,
                              const unsigned long long* w_ptrs, const unsigned long long* c_ptrs, hipStream_t s,
                              const int* a_rows = nullptr);

struct AttnArgs {
  const void* q; int ldq;   // bf16, row = token (b*S + s), head h at column h*D
  const void* k; int ldk;   // kv head g at column g*D
  const void* v; int ldv;
  void* o; int ldo;         // bf16 output, head h at column h*D
  int B, S, n_head, n_kv_head, D;
  float scale;
  int causal;
  int variant = 0;  // 0 auto; 1..11 fixed (waves, K/V stages, key split) — benchmarks/tuning
  // Sequence-chunked attention (context parallelism as a DAG): q holds Sq query rows per
  // batch at global positions q_off .. q_off+Sq-1; k/v hold S key rows per batch (positions
  // 0 .. S-1). Sq = 0 means Sq = S, q_off = 0 (ordinary self-attention).
  int Sq = 0;
  int q_off = 0;
  int flags = 0;  // bit 0: output stores write-through (sc1); bit 1: XCD-grouped blocks
  void* part = nullptr;  // variant 14: fp32 partials, attention_split_sizes() floats
  void* cnt = nullptr;   // variant 14: int32 tickets, zero before the first launch (self-resetting)
};
void launch_attention_fwd(const AttnArgs& a, hipStream_t s);
void attention_split_sizes(const AttnArgs& a, size_t* part_floats, size_t* counters);

// y = LN(x [+ r]) * w + b ; if r != nullptr and sum_out != nullptr, sum_out = x + r
void launch_layernorm(const void* x, const void* r, void* sum_out, const void* w, const void* b, void* y, int M,
                      int H, float eps, hipStream_t s);
void launch_rmsnorm(const void* x, const void* r, void* sum_out, const void* w, void* y, int M, int H, float eps,
                    hipStream_t s);

void launch_gelu(const void* x, void* y, int64_t n, hipStream_t s);
void launch_add(const void* a, const void* b, void* y, int64_t n, hipStream_t s);
void launch_swiglu(const void* gu, void* y, int M, int F, hipStream_t s);  // gu [M][2F] (gate|up)
void launch_embedding(const int32_t* tokens, const void* wte, const void* wpe, void* y, int M, int S, int H,
                      hipStream_t s, float* zbuf = nullptr, int zn = 0, float* stats = nullptr);
// in-place rotary embedding on the q and k head slices of a packed qkv row buffer
void launch_rope(void* qkv, int ld, int M, int S, int n_head, int n_kv_head, int D, int k_col, const float* cos_t,
                 const float* sin_t, hipStream_t s);

// MoE
void launch_moe_router(const void* logits, int M, int E, int topk, int32_t* topk_idx, float* topk_w,
                       hipStream_t s);
void launch_moe_align(const int32_t* topk_idx, int M, int topk, int E, int32_t* src_rows, int32_t* slot_of,
                      int32_t* offsets, hipStream_t s);
// router + align in one workgroup (M * topk <= kRouteMaxAssign): same outputs as the pair
constexpr int kRouteMaxAssign = 16384;
void launch_moe_route(const void* logits, int M, int E, int topk, int32_t* topk_idx, float* topk_w,
                      int32_t* src_rows, int32_t* slot_of, int32_t* offsets, hipStream_t s);
// router GEMM (logits = x Wg^T, bf16) + routing in one launch; false (nothing launched) when
// the shape is outside its limits (E * H <= 32768, M * max(k, E) <= kRouteMaxAssign, E even, E <= 16)
bool launch_moe_gate_route(const void* x, int ldx, const void* wg, int M, int H, int E, int topk, void* logits,
                           int* ticket, int32_t* topk_idx, float* topk_w, int32_t* src_rows, int32_t* slot_of,
                           int32_t* offsets, hipStream_t s);
void launch_moe_permute(const void* x, const int32_t* src_rows, void* out, int rows, int H, hipStream_t s);
// cross-request expert batch: per group g = (request req[g], expert expert[g]) the device-side
// row range of that request's routing (off[req]: int32 [E+1]) placed at base[req] — writes the
// groups' offsets [G+1] and the token row of every sorted row (a_rows) for one grouped launch
constexpr int kXbatchMaxReq = 16, kXbatchMaxGroups = 64;
struct XbatchIndexArgs {
  const int32_t* off[kXbatchMaxReq];
  int32_t base[kXbatchMaxReq];
  int32_t req[kXbatchMaxGroups];
  int32_t expert[kXbatchMaxGroups];
  int G;
  int32_t* offsets;
  int32_t* a_rows;
};
void launch_moe_xbatch_index(const XbatchIndexArgs& a, hipStream_t s);
// Expert-parallel capacity edges (fixed-size RCCL messages, parallel/executor.py): the rows a
// layer's routing sends to one expert GPU, packed (home rank) into / unpacked (expert GPU) from
// a [cap][H] buffer in expert-sorted order — experts in the listed order, each expert's rows in
// its sorted order. Rows past cap are not moved: the launch then sets ovf[flag] = 1 (and
// ovf[eflag[k]] for an expert whose own count exceeds ecap[k]: its compact output rows
// travel back in an edge of that capacity). No host sync: the counts are the device routing's.
constexpr int kMoePackMaxDest = 8, kMoePackMaxExp = 8;
struct MoePackDest {
  void* buf;                        // [cap][H] compact rows
  int cap, n_exp, flag;
  int experts[kMoePackMaxExp];
  int ecap[kMoePackMaxExp], eflag[kMoePackMaxExp];  // per expert: return-edge capacity / flag (-1: none)
};
struct MoePackArgs {
  MoePackDest d[kMoePackMaxDest];
  int n;
};
// unpack = 0: buf[c] = x[src[j]] (x: token rows); 1: x[j] = buf[c] (x: the expert-sorted rows)
void launch_moe_pack(const void* x, int H, const int32_t* src_rows, const int32_t* offsets, const MoePackArgs& a,
                     int32_t* ovf, int unpack, int max_rows, hipStream_t s);
void launch_moe_combine(const void* expert_out, const int32_t* slot_of, const float* weights, void* y, int M,
                        int topk, int H, const int32_t* range, hipStream_t s);
// X [rows][K] sorted by expert, offsets [E+1], W [E][N][K] -> Y [rows][N]
void launch_grouped_gemm(const void* X, const int32_t* offsets, const void* W, void* Y, int E, int N, int K,
                         int max_rows, int act, hipStream_t s);

// y[m] = r[m] + sum_j w[m,j] * expert_{idx[m,j]}[slot[m,j] - off[idx[m,j]]] over compact per-expert
// outputs whose base addresses are the device array eo_ptrs[E]; topk <= 8
// yn (optional, H <= 8192): also write norm(y) * nw (+ nb) for the next norm (nmode 1 LayerNorm, 2 RMSNorm)
void launch_moe_gather_combine(const unsigned long long* eo_ptrs, const int32_t* idx, const int32_t* slot_of,
                               const int32_t* off, const float* w, const void* r, void* y, int M, int topk, int H,
                               int E, hipStream_t s, void* yn = nullptr, const void* nw = nullptr,
                               const void* nb = nullptr, int nmode = 0, float neps = 1e-5f);

// dst (HBM) <- src (pinned host memory, device-accessible address); bytes % 16 == 0, both
// 16-byte aligned; at most `blocks` workgroups of 256 lanes pull over the host link
void launch_host_pull(const void* src, void* dst, int64_t bytes, int blocks, hipStream_t s);
void launch_delay(double us, hipStream_t s);

// GPT-2 MLP block in one launch (gemm_fused.hip): h = act1(LN(x) W1'^T + b1) (folded norm with
// handed-over row statistics), out = h W2^T + b2 + R (+ row statistics of out into stats_out)
// One-launch pre-norm attention block (attn_block.hip): QKV GEMM with a folded norm, causal
// MHA (head_dim 64), out-proj + bias + residual (+ next-norm row statistics), linked in-launch.
struct AttnBlockArgs {
  const void* x; int ldx;              // block input rows [M][H] (raw: the norm is folded)
  const void* w1; const void* b1;      // derived QKV weight [3H][H], bias' [3H] (or null)
  const float* colsum1;                // colsum(W') [3H]
  const float* ext_stats;              // (sum, sum of squares) of x's rows [M][2], from x's producer
  int ln_mode; float ln_eps;           // 1 LayerNorm, 2 RMSNorm
  void* qkv; int ldqkv;                // workspace [M][3H]
  void* o; int ldo;                    // workspace [M][H]
  const void* wo; const void* bo;      // out-proj [H][H], bias [H] (or null)
  const void* R; int ldr;              // residual [M][H]
  void* out; int ldout;                // block output [M][H]
  float* stats_out;                    // row statistics of out for the next folded norm (or null)
  int M, H, B, S, n_head;
  float scale;
  int* sync;                           // attn_block_sync_ints() ints, zero before the first launch
  int* err;                            // set when a poll exceeds spin_limit
  int spin_limit;
  unsigned long long* stamps = nullptr;  // diagnostic: [grid][4] (item, start, wait done, end) ticks
};
int attn_block_sync_ints(int M, int S, int B, int n_head);
bool attn_block_supported(int M, int H, int B, int S, int n_head, int n_kv_head, int D);
void launch_attn_block(const AttnBlockArgs& p, hipStream_t s);

struct MlpFusedArgs {
  const void* x;
  int ldx;
  const void* w1;
  int ldw1;
  const void* b1;
  const float* colsum1;
  const float* ext_stats;
  int ln_mode;
  float ln_eps;
  int act1;
  void* h;
  int ldh;
  const void* w2;
  int ldw2;
  const void* b2;
  const void* R;
  int ldr;
  void* out;
  int ldo;
  float* stats_out;
  int M, H, F, Hout;
  int* ready;  // [M / 64] arrival counters, zero before the launch (reset by the launch itself)
  int* done;   // [M / 64]
  int* err;    // set if a poll exceeded spin_limit
  int spin_limit;
  // before its poll, each workgroup DMAs its share of its fc2 weight panel (the panel is
  // shared by the XCD's workgroups of that column tile) so phase 2 finds it in the XCD's L2;
  // -1: DLS_MLP_PREFETCH (default on)
  int prefetch_w2 = -1;
};
bool mlp_fused_supported(int M, int H, int F, int Hout, int cus);
void launch_mlp_fused(const MlpFusedArgs& p, hipStream_t s);  // one wave spinning for ``us`` microseconds (loopback.cpp)
