// torch bindings for the hand-written HIP/CDNA4 kernels (module _dlsched_ops).
//
// Every op validates device / dtype / layout on the host before launching (a kernel
// that indexes past its operands can take the whole node down), launches on torch's
// current HIP stream (so the executor's stream and hipGraph capture apply), and
// allocates outputs through torch's caching allocator unless the caller passes `out`
// (the executor passes views into its HBM arena).
#include <cstdlib>

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// Split-K tile counters for the in-launch combine: one zeroed int32 pool per device (allocated
// on first use — the executor's eager warm-up step runs before any hipGraph capture), handed
// out round-robin so kernels in flight on other streams never share a counter; each tile's
// last arriver resets its counter, so a region is zero again whenever it is reused.
constexpr int64_t kSemPool = 1 << 20;
int* split_k_counters(const at::Tensor& like, int64_t n) {
  // heap-held and never freed: a static tensor's destructor would run after the HIP runtime
  // and the caching allocator have been torn down at interpreter exit
  static at::Tensor* pool = new at::Tensor[64];
  static int64_t next[64];
  const int d = like.get_device();
  TORCH_CHECK(d >= 0 && d < 64 && n <= kSemPool, "split-K counters");
  if (!pool[d].defined()) pool[d] = at::zeros({kSemPool}, like.options().dtype(at::kInt));
  n = (n + 63) / 64 * 64;
  if (next[d] + n > kSemPool) next[d] = 0;
  int* p = pool[d].data_ptr<int>() + next[d];
  next[d] += n;
  return p;
}
const bool kSplitKFixup = [] {
  const char* e = std::getenv("DLS_SPLITK_FIXUP");
  return !(e && e[0] == '0');
}();

void check_bf16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}

// 2-D view [rows][cols] with unit column stride and 16-B aligned rows
void check_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.stride(1) == 1, name, " must have contiguous rows");
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8 elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

at::Tensor as2d(const at::Tensor& t) { return t.dim() == 2 ? t : t.reshape({-1, t.size(-1)}); }

// splitk: 0 auto (LDS-DMA path), otherwise forced.
// config: -1 auto, 0..gemm_glds_num_configs()-1 LDS-DMA kernel, >= kRegStage register-staged kernel.
// act ACT_SWIGLU: W rows interleave gate/up blocks of 16 (see common.h); the output is N/2 wide.
// rows (int32[2] on device): only rows [rows[0], rows[1]) of A / out take part (MoE expert ranges).
constexpr int64_t kRegStage = 100;

at::Tensor gemm(const at::Tensor& a_in, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                const c10::optional<at::Tensor>& residual, int64_t act, double alpha,
                const c10::optional<at::Tensor>& out, int64_t config, int64_t splitk,
                const c10::optional<at::Tensor>& ln_colsum, int64_t ln_mode, double ln_eps,
                const c10::optional<at::Tensor>& rows, bool compact_rows,
                const c10::optional<at::Tensor>& rope_cos, const c10::optional<at::Tensor>& rope_sin, int64_t rope_S,
                int64_t rope_D, int64_t rope_cols, const c10::optional<at::Tensor>& stats_out,
                const c10::optional<at::Tensor>& ext_stats, const c10::optional<at::Tensor>& norm_out,
                const c10::optional<at::Tensor>& norm_w, const c10::optional<at::Tensor>& norm_b, int64_t norm_mode,
                double norm_eps, int64_t stream_pol) {
  check_bf16(a_in, "A");
  check_bf16(w, "W");
  at::Tensor a = as2d(a_in);
  check_rows(a, "A");
  check_rows(w, "W");
  const int64_t M = a.size(0), K = a.size(1), N = w.size(0);
  const bool swiglu = act == kActSwiglu;
  const int64_t NO = swiglu ? N / 2 : N;
  TORCH_CHECK(w.size(1) == K, "W must be [N][K] with K = ", K, ", got ", w.sizes());
  TORCH_CHECK(K % 8 == 0, "K must be a multiple of 8");
  TORCH_CHECK(!swiglu || (N % 32 == 0 && K % 64 == 0 && !residual.has_value()),
              "SwiGLU epilogue needs N % 32 == 0, K % 64 == 0 and no residual");
  at::Tensor c;
  if (out.has_value()) {
    c = as2d(*out);
    check_bf16(c, "out");
    TORCH_CHECK((c.size(0) == M || (compact_rows && c.size(0) <= M)) && c.size(1) == NO && c.stride(1) == 1,
                "out must be [M][N_out] (or fewer rows with compact_rows)");
  } else {
    c = at::empty({M, NO}, a.options());
  }
  const void* bptr = nullptr;
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N, "bias must be contiguous [N]");
    bptr = bias->data_ptr();
  }
  const void* rptr = nullptr;
  int ldr = 0;
  if (residual.has_value()) {
    at::Tensor r = as2d(*residual);
    check_bf16(r, "residual");
    TORCH_CHECK(r.size(0) == M && r.size(1) == N && r.stride(1) == 1, "residual must be [M][N]");
    rptr = r.data_ptr();
    ldr = (int)r.stride(0);
  }
  const int* rowp = nullptr;
  if (rows.has_value()) {
    TORCH_CHECK(rows->scalar_type() == at::kInt && rows->numel() == 2 && rows->is_contiguous() &&
                    rows->device() == a.device(),
                "rows must be a contiguous int32[2] device tensor");
    TORCH_CHECK(K % 64 == 0 && ln_mode == 0, "row-ranged GEMM needs K % 64 == 0 and no folded norm");
    rowp = rows->data_ptr<int>();
  }
  if (M == 0 || N == 0) return c;
  GemmArgs g{a.data_ptr(), (int)a.stride(0), w.data_ptr(), (int)w.stride(0), c.data_ptr(), (int)c.stride(0),
             bptr, rptr, ldr, (int)M, (int)N, (int)K, (int)act, (float)alpha, -1,
             (compact_rows && rows.has_value()) ? (int)c.size(0) : 0};
  g.stream_pol = (int)stream_pol;
  // post-norm for the next (unfolded) norm: a split-K launch writes it from its row-owning
  // reduce; every other path runs the norm kernel on the output right after the GEMM
  at::Tensor y_n;
  if (norm_out.has_value()) {
    TORCH_CHECK(norm_mode == 1 || norm_mode == 2, "norm_mode: 1 LayerNorm, 2 RMSNorm");
    TORCH_CHECK(!swiglu && !rows.has_value() && c.is_contiguous(), "post-norm needs a full, contiguous output");
    y_n = as2d(*norm_out);
    check_bf16(y_n, "norm_out");
    TORCH_CHECK(y_n.is_contiguous() && y_n.size(0) == M && y_n.size(1) == N, "norm_out must be contiguous [M][N]");
    TORCH_CHECK(norm_w.has_value() && norm_w->is_contiguous() && norm_w->numel() == N, "norm_w [N]");
    check_bf16(*norm_w, "norm_w");
    TORCH_CHECK(norm_mode == 2 || (norm_b.has_value() && norm_b->is_contiguous() && norm_b->numel() == N),
                "LayerNorm post-norm needs norm_b [N]");
    g.norm_out = y_n.data_ptr();
    g.ldn = (int)N;
    g.norm_w = norm_w->data_ptr();
    g.norm_b = norm_mode == 1 ? norm_b->data_ptr() : nullptr;
    g.norm_mode = (int)norm_mode;
    g.norm_eps = (float)norm_eps;
  }
  auto post_norm = [&](bool done) {
    if (!norm_out.has_value() || done) return;
    if (norm_mode == 2)
      launch_rmsnorm(c.data_ptr(), nullptr, nullptr, g.norm_w, y_n.data_ptr(), (int)M, (int)N, (float)norm_eps,
                     cur_stream());
    else
      launch_layernorm(c.data_ptr(), nullptr, nullptr, g.norm_w, g.norm_b, y_n.data_ptr(), (int)M, (int)N,
                       (float)norm_eps, cur_stream());
  };
  TORCH_CHECK(!compact_rows || (rows.has_value() && !residual.has_value()), "compact_rows needs rows and no residual");
  auto check_stats = [&](const at::Tensor& t, const char* name) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == 2 * M, name,
                " must be a contiguous fp32 [M][2] GPU tensor");
  };
  if (stats_out.has_value()) {
    check_stats(*stats_out, "stats_out");
    TORCH_CHECK(!swiglu && !rows.has_value(), "row statistics are emitted by plain (non-SwiGLU, full-row) GEMMs");
    g.stats_out = stats_out->data_ptr<float>();
  }
  if (ext_stats.has_value()) {
    check_stats(*ext_stats, "ext_stats");
    TORCH_CHECK(ln_mode != 0, "ext_stats needs ln_mode (1 LayerNorm, 2 RMSNorm) and ln_colsum");
    g.ext_stats = ext_stats->data_ptr<float>();
  }
  if (rope_cols > 0) {
    TORCH_CHECK(rope_cos.has_value() && rope_sin.has_value() && rope_cos->scalar_type() == at::kFloat &&
                    rope_sin->scalar_type() == at::kFloat && rope_cos->is_contiguous() && rope_sin->is_contiguous() &&
                    rope_cos->is_cuda() && rope_sin->is_cuda() &&
                    rope_cos->numel() >= rope_S * rope_D / 2 && rope_sin->numel() >= rope_S * rope_D / 2,
                "RoPE epilogue: cos/sin fp32 [S][D/2]");
    TORCH_CHECK(rope_D % 4 == 0 && rope_cols % rope_D == 0 && rope_cols <= N && !swiglu && K % 64 == 0 &&
                    !rows.has_value() && act == 0,
                "RoPE epilogue: D % 4 == 0, whole heads, LDS-DMA kernel, no activation / SwiGLU / row range");
    g.rope = RopeArgs{rope_cos->data_ptr<float>(), rope_sin->data_ptr<float>(), (int)rope_S, (int)rope_D,
                      (int)rope_cols};
    if (config >= kRegStage) config = -1;
  }
  const bool glds_ok = (K % 64 == 0);
  const float* csp = nullptr;
  if (ln_mode != 0) {
    TORCH_CHECK(glds_ok, "fused norm-GEMM needs K % 64 == 0");
    TORCH_CHECK(ln_colsum.has_value() && ln_colsum->scalar_type() == at::kFloat && ln_colsum->is_contiguous() &&
                    ln_colsum->numel() == N,
                "fused norm-GEMM needs fp32 ln_colsum [N]");
    csp = ln_colsum->data_ptr<float>();
  }
  if (ln_mode != 0 || swiglu || rowp || stats_out.has_value()) {
    TORCH_CHECK(glds_ok, "this epilogue needs the LDS-DMA kernel (K % 64 == 0)");
    if (config >= kRegStage) config = -1;  // these epilogues live in the LDS-DMA kernel only
  }
  if (config >= kRegStage || !glds_ok) {
    g.config = config >= kRegStage ? (int)(config - kRegStage) : -1;
    launch_gemm_bf16(g, cur_stream());
    post_norm(false);
    return c;
  }
  int cfg = (int)config, sk = (int)splitk;
  if (cfg < 0 || sk <= 0) {
    int acfg, ask;
    gemm_glds_pick((int)M, (int)N, (int)K, &acfg, &ask);
    if (cfg < 0) cfg = acfg;
    if (sk <= 0) sk = ask;
  }
  TORCH_CHECK((cfg & (kGemmPersist - 1)) < gemm_glds_num_configs() && cfg < 2 * kGemmPersist, "unknown GEMM config ", cfg);
  TORCH_CHECK(K % gemm_glds_kstep(cfg) == 0, "GEMM config ", cfg, " needs K % ", gemm_glds_kstep(cfg), " == 0");
  const bool split_ok = (N % 8 == 0) && (c.stride(0) % 8 == 0) && (ldr % 8 == 0) &&
                        K % (gemm_glds_kstep(cfg) * sk) == 0 &&
                        (!swiglu || N % 32 == 0);
  if (!split_ok || (ln_mode != 0 && !ext_stats.has_value())) sk = 1;
  at::Tensor ws;
  if (sk > 1) {
    ws = at::empty({(int64_t)gemm_glds_workspace_bytes((int)M, (int)N, sk) / 4}, a.options().dtype(at::kFloat));
    // (a post-norm wants the row-owning reduce kernel, not the in-launch combine)
    if (kSplitKFixup && !rowp && !norm_out.has_value())
      g.tile_sem = split_k_counters(a, (M + 63) / 64 * ((N + 63) / 64));
  }
  post_norm(launch_gemm_glds(g, cfg, sk, sk > 1 ? ws.data_ptr() : nullptr, cur_stream(), csp, (int)ln_mode,
                             (float)ln_eps, rowp));
  return c;
}

at::Tensor attention(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t B, int64_t S,
                     int64_t n_head, int64_t n_kv_head, int64_t head_dim, bool causal, double scale,
                     const c10::optional<at::Tensor>& out, int64_t variant, int64_t Sq, int64_t q_off,
                     int64_t flags) {
  if (Sq <= 0) Sq = S;
  TORCH_CHECK(q_off >= 0 && (!causal || q_off + Sq <= S), "query chunk must lie inside the key range");
  for (auto* p : {&q, &k, &v}) {
    check_bf16(*p, "qkv");
    check_rows(*p, "qkv");
    TORCH_CHECK(p->size(0) == B * (p == &q ? Sq : S), "q must have B*Sq rows and k/v B*S rows");
  }
  TORCH_CHECK(head_dim == 64 || head_dim == 128, "head_dim must be 64 or 128");
  TORCH_CHECK(n_head % n_kv_head == 0, "n_head must be a multiple of n_kv_head");
  TORCH_CHECK(q.size(1) >= n_head * head_dim && k.size(1) >= n_kv_head * head_dim &&
                  v.size(1) >= n_kv_head * head_dim,
              "q/k/v column extent too small for the head layout");
  at::Tensor o = out.has_value() ? as2d(*out) : at::empty({B * Sq, n_head * head_dim}, q.options());
  check_rows(o, "out");
  TORCH_CHECK(o.size(0) == B * Sq && o.size(1) >= n_head * head_dim, "out must be [B*Sq, >= n_head*head_dim]");
  AttnArgs a{q.data_ptr(), (int)q.stride(0), k.data_ptr(), (int)k.stride(0), v.data_ptr(), (int)v.stride(0),
             o.data_ptr(), (int)o.stride(0), (int)B, (int)S, (int)n_head, (int)n_kv_head, (int)head_dim,
             (float)scale, causal ? 1 : 0, (int)variant, (int)Sq, (int)q_off,
             // write-through stores use 32-bit buffer offsets: not for outputs of 2 GB or more
             (int)(o.numel() * 2 < (1ll << 31) ? flags : flags & ~1)};
  at::Tensor part;
  if (variant == 14) {  // one key tile per block: fp32 partials + self-resetting tickets
    size_t pf = 0, nc = 0;
    attention_split_sizes(a, &pf, &nc);
    part = at::empty({(int64_t)pf}, q.options().dtype(at::kFloat));
    a.part = part.data_ptr();
    a.cnt = split_k_counters(q, (int64_t)nc);
  }
  launch_attention_fwd(a, cur_stream());
  return o;
}

std::vector<at::Tensor> norm(const at::Tensor& x_in, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                             double eps, const c10::optional<at::Tensor>& residual, bool rms,
                             const c10::optional<at::Tensor>& out, const c10::optional<at::Tensor>& sum_out) {
  check_bf16(x_in, "x");
  at::Tensor x = as2d(x_in).contiguous();
  const int64_t M = x.size(0), H = x.size(1);
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "hidden size must be a multiple of 8 and <= 8192");
  check_bf16(w, "weight");
  TORCH_CHECK(w.is_contiguous() && w.numel() == H, "weight must be contiguous [H]");
  if (b.has_value()) {
    check_bf16(*b, "bias");
    TORCH_CHECK(b->is_contiguous() && b->numel() == H, "bias must be contiguous [H]");
  }
  at::Tensor y = out.has_value() ? as2d(*out) : at::empty({M, H}, x.options());
  TORCH_CHECK(y.is_contiguous(), "out must be contiguous");
  at::Tensor r, s;
  if (residual.has_value()) {
    r = as2d(*residual).contiguous();
    check_bf16(r, "residual");
    TORCH_CHECK(r.sizes() == x.sizes(), "residual must match x");
    s = sum_out.has_value() ? as2d(*sum_out) : at::empty({M, H}, x.options());
    TORCH_CHECK(s.is_contiguous(), "sum_out must be contiguous");
  }
  if (M == 0) return {y, s};
  if (rms)
    launch_rmsnorm(x.data_ptr(), r.defined() ? r.data_ptr() : nullptr, s.defined() ? s.data_ptr() : nullptr,
                   w.data_ptr(), y.data_ptr(), (int)M, (int)H, (float)eps, cur_stream());
  else
    launch_layernorm(x.data_ptr(), r.defined() ? r.data_ptr() : nullptr, s.defined() ? s.data_ptr() : nullptr,
                     w.data_ptr(), b.has_value() ? b->data_ptr() : nullptr, y.data_ptr(), (int)M, (int)H,
                     (float)eps, cur_stream());
  return {y, s};
}

at::Tensor gelu(const at::Tensor& x, const c10::optional<at::Tensor>& out) {
  check_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "x must be contiguous with numel % 8 == 0");
  at::Tensor y = out.has_value() ? *out : at::empty_like(x);
  TORCH_CHECK(y.is_contiguous() && y.numel() == x.numel(), "out mismatch");
  launch_gelu(x.data_ptr(), y.data_ptr(), x.numel(), cur_stream());
  return y;
}

at::Tensor add(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& out) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous() && a.numel() == b.numel() && a.numel() % 8 == 0,
              "add operands must be contiguous, equal-sized, numel % 8 == 0");
  at::Tensor y = out.has_value() ? *out : at::empty_like(a);
  TORCH_CHECK(y.is_contiguous() && y.numel() == a.numel(), "out mismatch");
  launch_add(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), cur_stream());
  return y;
}

at::Tensor swiglu(const at::Tensor& gu_in, const c10::optional<at::Tensor>& out) {
  check_bf16(gu_in, "gate_up");
  at::Tensor gu = as2d(gu_in).contiguous();
  const int64_t M = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(gu.size(1) % 16 == 0, "gate_up width must be 2F with F % 8 == 0");
  at::Tensor y = out.has_value() ? as2d(*out) : at::empty({M, F}, gu.options());
  TORCH_CHECK(y.is_contiguous() && y.size(0) == M && y.size(1) == F, "out mismatch");
  launch_swiglu(gu.data_ptr(), y.data_ptr(), (int)M, (int)F, cur_stream());
  return y;
}

// GPT-2 MLP block as one launch (gemm_fused.hip): h = GELU(LN(x) W1'^T + b1') with the folded
// LayerNorm's statistics handed over (ext_stats), out = h W2^T + b2 + residual (+ stats_out).
// sync: int32 [2 * M / 64 + 1] zeroed once (arrival / consumer counters, error word).
int64_t mlp_fused_cus() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus;
}

bool mlp_fused_ok(int64_t M, int64_t H, int64_t F, int64_t Hout) {
  return mlp_fused_supported((int)M, (int)H, (int)F, (int)Hout, (int)mlp_fused_cus());
}

void mlp_fused(const at::Tensor& x_in, const at::Tensor& w1, const c10::optional<at::Tensor>& b1,
               const at::Tensor& colsum1, const at::Tensor& ext_stats, int64_t ln_mode, double eps, int64_t act1,
               const at::Tensor& h_in, const at::Tensor& w2, const c10::optional<at::Tensor>& b2,
               const at::Tensor& res_in, const at::Tensor& out_in, const c10::optional<at::Tensor>& stats_out,
               const at::Tensor& sync, int64_t spin_limit) {
  at::Tensor x = as2d(x_in), h = as2d(h_in), r = as2d(res_in), o = as2d(out_in);
  for (auto* t : {&x, &h, &r, &o}) check_bf16(*t, "mlp_fused operand");
  check_bf16(w1, "w1");
  check_bf16(w2, "w2");
  for (auto* t : {&x, &h, &r, &o}) check_rows(*t, "mlp_fused operand");
  check_rows(w1, "w1");
  check_rows(w2, "w2");
  const int64_t M = x.size(0), H = x.size(1), F = w1.size(0), Hout = w2.size(0);
  TORCH_CHECK(w1.size(1) == H && w2.size(1) == F && h.size(0) == M && h.size(1) == F && r.size(0) == M &&
                  r.size(1) == Hout && o.size(0) == M && o.size(1) == Hout,
              "mlp_fused: x [M][H], w1 [F][H], h [M][F], w2 [Hout][F], residual / out [M][Hout]");
  TORCH_CHECK(mlp_fused_ok(M, H, F, Hout), "mlp_fused: shape not supported by the one-launch MLP (M ", M, ", H ", H,
              ", F ", F, ", Hout ", Hout, ")");
  TORCH_CHECK(ln_mode == 1 || ln_mode == 2, "mlp_fused: ln_mode 1 LayerNorm, 2 RMSNorm");
  auto f32 = [&](const at::Tensor& t, int64_t n, const char* name) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, name,
                " must be a contiguous fp32 GPU tensor of ", n, " elements");
  };
  f32(colsum1, F, "colsum1");
  f32(ext_stats, 2 * M, "ext_stats");
  if (stats_out.has_value()) f32(*stats_out, 2 * M, "stats_out");
  for (auto* b : {&b1, &b2})
    if (b->has_value()) {
      check_bf16(**b, "bias");
      TORCH_CHECK((*b)->is_contiguous(), "bias must be contiguous");
    }
  TORCH_CHECK(!b1.has_value() || b1->numel() == F, "b1 must be [F]");
  TORCH_CHECK(!b2.has_value() || b2->numel() == Hout, "b2 must be [Hout]");
  const int64_t rb = M / 64;
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == at::kInt && sync.is_contiguous() && sync.numel() >= 2 * rb + 1,
              "sync must be a zeroed int32 GPU tensor of >= 2 * M / 64 + 1 elements");
  MlpFusedArgs p{x.data_ptr(), (int)x.stride(0), w1.data_ptr(), (int)w1.stride(0),
                 b1.has_value() ? b1->data_ptr() : nullptr, colsum1.data_ptr<float>(), ext_stats.data_ptr<float>(),
                 (int)ln_mode, (float)eps, (int)act1, h.data_ptr(), (int)h.stride(0), w2.data_ptr(),
                 (int)w2.stride(0), b2.has_value() ? b2->data_ptr() : nullptr, r.data_ptr(), (int)r.stride(0),
                 o.data_ptr(), (int)o.stride(0), stats_out.has_value() ? stats_out->data_ptr<float>() : nullptr,
                 (int)M, (int)H, (int)F, (int)Hout, sync.data_ptr<int>(), sync.data_ptr<int>() + rb,
                 sync.data_ptr<int>() + 2 * rb, (int)spin_limit};
  launch_mlp_fused(p, cur_stream());
}

at::Tensor embedding(const at::Tensor& tokens, const at::Tensor& wte, const c10::optional<at::Tensor>& wpe, int64_t S,
                     const c10::optional<at::Tensor>& out, const c10::optional<at::Tensor>& zero,
                     const c10::optional<at::Tensor>& stats) {
  TORCH_CHECK(tokens.is_cuda() && tokens.scalar_type() == at::kInt && tokens.is_contiguous(),
              "tokens must be contiguous int32 on the GPU");
  check_bf16(wte, "wte");
  TORCH_CHECK(wte.is_contiguous(), "wte must be contiguous");
  const int64_t M = tokens.numel(), H = wte.size(1);
  TORCH_CHECK(H % 8 == 0, "hidden size must be a multiple of 8");
  if (wpe.has_value()) {
    check_bf16(*wpe, "wpe");
    TORCH_CHECK(wpe->is_contiguous() && wpe->size(1) == H && wpe->size(0) >= S, "wpe must be [>=S][H]");
  }
  at::Tensor y = out.has_value() ? as2d(*out) : at::empty({M, H}, wte.options());
  TORCH_CHECK(y.is_contiguous() && y.size(0) == M && y.size(1) == H, "out mismatch");
  float* zb = nullptr;
  int zn = 0;
  if (zero.has_value()) {
    TORCH_CHECK(zero->is_cuda() && zero->scalar_type() == at::kFloat && zero->is_contiguous(),
                "zero must be a contiguous fp32 GPU tensor");
    zb = zero->data_ptr<float>();
    zn = (int)zero->numel();
  }
  float* st = nullptr;
  if (stats.has_value()) {
    TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kFloat && stats->is_contiguous() &&
                    stats->numel() >= 2 * M,
                "stats must be a contiguous fp32 GPU tensor of >= 2 * rows");
    st = stats->data_ptr<float>();
    if (zb) {  // the kernel zeroes zero[] while other workgroups write stats[]: disjoint only
      const float* z0 = zb;
      const float* s0 = st;
      TORCH_CHECK(s0 + 2 * M <= z0 || z0 + zn <= s0, "stats must not overlap the zeroed buffer");
    }
  }
  launch_embedding(tokens.data_ptr<int32_t>(), wte.data_ptr(), wpe.has_value() ? wpe->data_ptr() : nullptr,
                   y.data_ptr(), (int)M, (int)S, (int)H, cur_stream(), zb, zn, st);
  return y;
}

void rope_(at::Tensor& qkv, int64_t S, int64_t n_head, int64_t n_kv_head, int64_t head_dim, int64_t k_col,
           const at::Tensor& cos_t, const at::Tensor& sin_t) {
  check_bf16(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "qkv must be a 2-D row buffer");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.numel() >= S * head_dim / 2,
              "cos/sin tables must be contiguous fp32 [S][D/2]");
  TORCH_CHECK(k_col + n_kv_head * head_dim <= qkv.size(1) && n_head * head_dim <= qkv.size(1), "head layout");
  TORCH_CHECK(head_dim % 16 == 0 && k_col % 8 == 0 && qkv.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0,
              "vectorised RoPE needs head_dim % 16 == 0 and 16-B aligned rows / k columns");
  launch_rope(qkv.data_ptr(), (int)qkv.stride(0), (int)qkv.size(0), (int)S, (int)n_head, (int)n_kv_head,
              (int)head_dim, (int)k_col, cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), cur_stream());
}

std::vector<at::Tensor> moe_router(const at::Tensor& logits, int64_t topk) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits must be contiguous [M][E]");
  const int64_t M = logits.size(0), E = logits.size(1);
  TORCH_CHECK(E <= 64 && topk >= 1 && topk <= 8 && topk <= E, "router supports E <= 64, 1 <= topk <= min(8, E)");
  auto idx = at::empty({M, topk}, logits.options().dtype(at::kInt));
  auto w = at::empty({M, topk}, logits.options().dtype(at::kFloat));
  launch_moe_router(logits.data_ptr(), (int)M, (int)E, (int)topk, idx.data_ptr<int32_t>(), w.data_ptr<float>(),
                    cur_stream());
  return {idx, w};
}

std::vector<at::Tensor> moe_align(const at::Tensor& idx, int64_t E) {
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kInt && idx.dim() == 2 && idx.is_contiguous(),
              "topk_idx must be contiguous int32 [M][k]");
  const int64_t M = idx.size(0), k = idx.size(1);
  auto opt = idx.options();
  auto src = at::empty({M * k}, opt), slot = at::empty({M * k}, opt), off = at::empty({E + 1}, opt);
  launch_moe_align(idx.data_ptr<int32_t>(), (int)M, (int)k, (int)E, src.data_ptr<int32_t>(),
                   slot.data_ptr<int32_t>(), off.data_ptr<int32_t>(), cur_stream());
  return {src, slot, off};
}

// router + align in ONE launch (route_kernel): idx, w, src_rows, slot_of, offsets
std::vector<at::Tensor> moe_route(const at::Tensor& logits, int64_t topk) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits must be contiguous [M][E]");
  const int64_t M = logits.size(0), E = logits.size(1);
  TORCH_CHECK(E <= 64 && topk >= 1 && topk <= 8 && topk <= E, "router supports E <= 64, 1 <= topk <= min(8, E)");
  TORCH_CHECK(M * topk <= kRouteMaxAssign, "fused routing holds at most ", kRouteMaxAssign, " assignments");
  auto iopt = logits.options().dtype(at::kInt);
  auto idx = at::empty({M, topk}, iopt);
  auto w = at::empty({M, topk}, logits.options().dtype(at::kFloat));
  auto src = at::empty({M * topk}, iopt), slot = at::empty({M * topk}, iopt), off = at::empty({E + 1}, iopt);
  launch_moe_route(logits.data_ptr(), (int)M, (int)E, (int)topk, idx.data_ptr<int32_t>(), w.data_ptr<float>(),
                   src.data_ptr<int32_t>(), slot.data_ptr<int32_t>(), off.data_ptr<int32_t>(), cur_stream());
  return {idx, w, src, slot, off};
}

// router GEMM + routing in ONE launch (gate_route_kernel): logits (bf16 [M][E], written to
// `logits`) and idx, w, src_rows, slot_of, offsets; an empty list when the shape is outside
// the kernel's limits (the caller then runs the GEMM and moe_route)
std::vector<at::Tensor> moe_gate_route(const at::Tensor& x, const at::Tensor& wg, int64_t topk, at::Tensor& logits) {
  check_bf16(x, "x");
  check_bf16(wg, "router weight");
  check_bf16(logits, "logits");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && wg.dim() == 2 && wg.is_contiguous() && wg.size(1) == x.size(1),
              "x [M][H] (rows contiguous), router weight contiguous [E][H]");
  const int64_t M = x.size(0), H = x.size(1), E = wg.size(0);
  TORCH_CHECK(logits.is_contiguous() && logits.numel() == M * E, "logits must be contiguous [M][E]");
  TORCH_CHECK(topk >= 1 && topk <= 8 && topk <= E, "1 <= topk <= min(8, E)");
  auto iopt = x.options().dtype(at::kInt);
  auto idx = at::empty({M, topk}, iopt);
  auto w = at::empty({M, topk}, x.options().dtype(at::kFloat));
  auto src = at::empty({M * topk}, iopt), slot = at::empty({M * topk}, iopt), off = at::empty({E + 1}, iopt);
  int* ticket = split_k_counters(x, 1);
  if (!launch_moe_gate_route(x.data_ptr(), (int)x.stride(0), wg.data_ptr(), (int)M, (int)H, (int)E, (int)topk,
                             logits.data_ptr(), ticket, idx.data_ptr<int32_t>(), w.data_ptr<float>(),
                             src.data_ptr<int32_t>(), slot.data_ptr<int32_t>(), off.data_ptr<int32_t>(), cur_stream()))
    return {};
  return {idx, w, src, slot, off};
}

at::Tensor moe_permute(const at::Tensor& x, const at::Tensor& src_rows, const c10::optional<at::Tensor>& out_) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0, "x must be contiguous [M][H]");
  TORCH_CHECK(src_rows.scalar_type() == at::kInt && src_rows.is_contiguous(), "src_rows must be int32");
  at::Tensor out;
  if (out_.has_value()) {
    out = *out_;
    check_bf16(out, "out");
    TORCH_CHECK(out.is_contiguous() && out.dim() == 2 && out.size(0) == src_rows.numel() && out.size(1) == x.size(1),
                "out must be contiguous [rows][H]");
  } else {
    out = at::empty({src_rows.numel(), x.size(1)}, x.options());
  }
  launch_moe_permute(x.data_ptr(), src_rows.data_ptr<int32_t>(), out.data_ptr(), (int)src_rows.numel(),
                     (int)x.size(1), cur_stream());
  return out;
}

// Expert-parallel capacity edges (kernels.h MoePackArgs): pack (unpack = false) the routed rows
// of each destination into its [cap][H] buffer, or unpack (true) a received buffer into the
// expert-sorted rows x. ovf: int32 flags (set to 1 where a count exceeded its capacity).
void moe_pack(const at::Tensor& x, const at::Tensor& src_rows, const at::Tensor& offsets,
              const std::vector<at::Tensor>& bufs, const std::vector<int64_t>& caps,
              const std::vector<std::vector<int64_t>>& experts, const std::vector<int64_t>& flags,
              const std::vector<std::vector<int64_t>>& ecaps, const std::vector<std::vector<int64_t>>& eflags,
              at::Tensor& ovf, bool unpack) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0, "x must be contiguous [rows][H], H % 8 == 0");
  TORCH_CHECK(src_rows.scalar_type() == at::kInt && offsets.scalar_type() == at::kInt && src_rows.is_contiguous() &&
                  offsets.is_contiguous() && src_rows.is_cuda() && offsets.is_cuda(),
              "src_rows / offsets: contiguous int32 GPU tensors");
  TORCH_CHECK(ovf.scalar_type() == at::kInt && ovf.is_cuda() && ovf.is_contiguous(), "ovf: int32 GPU tensor");
  const size_t n = bufs.size();
  TORCH_CHECK(n >= 1 && n <= (size_t)kMoePackMaxDest && caps.size() == n && experts.size() == n &&
                  flags.size() == n && ecaps.size() == n && eflags.size() == n,
              "moe_pack: 1..", kMoePackMaxDest, " destinations, one entry each");
  const int64_t H = x.size(1), E = offsets.numel() - 1;
  MoePackArgs a{};
  a.n = (int)n;
  int max_rows = 0;
  for (size_t d = 0; d < n; ++d) {
    check_bf16(bufs[d], "buf");
    TORCH_CHECK(bufs[d].is_contiguous() && bufs[d].numel() >= caps[d] * H, "buf ", d, " must hold cap x H elements");
    TORCH_CHECK(experts[d].size() >= 1 && experts[d].size() <= (size_t)kMoePackMaxExp &&
                    ecaps[d].size() == experts[d].size() && eflags[d].size() == experts[d].size(),
                "moe_pack: 1..", kMoePackMaxExp, " experts per destination");
    TORCH_CHECK(flags[d] < ovf.numel(), "flag index out of range");
    a.d[d].buf = bufs[d].data_ptr();
    a.d[d].cap = (int)caps[d];
    a.d[d].n_exp = (int)experts[d].size();
    a.d[d].flag = (int)flags[d];
    for (size_t k = 0; k < experts[d].size(); ++k) {
      TORCH_CHECK(experts[d][k] >= 0 && experts[d][k] < E, "expert id out of range");
      TORCH_CHECK(eflags[d][k] < ovf.numel(), "expert flag index out of range");
      a.d[d].experts[k] = (int)experts[d][k];
      a.d[d].ecap[k] = (int)ecaps[d][k];
      a.d[d].eflag[k] = (int)eflags[d][k];
    }
    max_rows = std::max(max_rows, (int)caps[d]);
  }
  if (unpack) TORCH_CHECK(x.size(0) >= src_rows.numel(), "unpack: x must hold the expert-sorted rows");
  launch_moe_pack(x.data_ptr(), (int)H, src_rows.data_ptr<int32_t>(), offsets.data_ptr<int32_t>(), a,
                  ovf.data_ptr<int32_t>(), unpack ? 1 : 0, max_rows, cur_stream());
}

// offs: each request's routing offsets (int32 [E+1], on the GPU); groups g: (reqs[g], experts[g]);
// bases[q]: row of request q's expert-sorted block in the batch's token matrix
void moe_xbatch_index(const std::vector<at::Tensor>& offs, const std::vector<int64_t>& reqs,
                      const std::vector<int64_t>& experts, const std::vector<int64_t>& bases, at::Tensor& offsets,
                      at::Tensor& a_rows) {
  const int Q = (int)offs.size(), G = (int)reqs.size();
  TORCH_CHECK(Q >= 1 && Q <= kXbatchMaxReq && (int)bases.size() == Q, "1..", kXbatchMaxReq, " requests, one base each");
  TORCH_CHECK(G >= 1 && G <= kXbatchMaxGroups && (int)experts.size() == G, "1..", kXbatchMaxGroups, " groups");
  TORCH_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.numel() == G + 1, "offsets int32 [G+1]");
  TORCH_CHECK(a_rows.is_cuda() && a_rows.scalar_type() == at::kInt && a_rows.is_contiguous(), "a_rows int32");
  XbatchIndexArgs a{};
  int64_t E = -1;
  for (int q = 0; q < Q; ++q) {
    TORCH_CHECK(offs[q].is_cuda() && offs[q].scalar_type() == at::kInt && offs[q].is_contiguous(),
                "routing offsets: int32 on the GPU");
    TORCH_CHECK(E < 0 || offs[q].numel() == E + 1, "every request routes over the same experts");
    E = offs[q].numel() - 1;
    a.off[q] = offs[q].data_ptr<int32_t>();
    a.base[q] = (int32_t)bases[q];
  }
  for (int g = 0; g < G; ++g) {
    TORCH_CHECK(reqs[g] >= 0 && reqs[g] < Q && experts[g] >= 0 && experts[g] < E, "group (request, expert) range");
    a.req[g] = (int32_t)reqs[g];
    a.expert[g] = (int32_t)experts[g];
  }
  // a_rows holds every group's rows: the caller sizes it to the requests' blocks (the device
  // counts of distinct (request, expert) pairs never exceed their requests' sorted orders)
  a.G = G;
  a.offsets = offsets.data_ptr<int32_t>();
  a.a_rows = a_rows.data_ptr<int32_t>();
  launch_moe_xbatch_index(a, cur_stream());
}

at::Tensor moe_combine(const at::Tensor& eo, const at::Tensor& slot_of, const at::Tensor& w,
                       const c10::optional<at::Tensor>& range, const c10::optional<at::Tensor>& out) {
  check_bf16(eo, "expert_out");
  TORCH_CHECK(eo.dim() == 2 && eo.is_contiguous() && eo.size(1) % 8 == 0, "expert_out must be contiguous [R][H]");
  TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kFloat && w.is_contiguous(), "weights must be fp32 [M][k]");
  TORCH_CHECK(slot_of.numel() == w.numel() && slot_of.scalar_type() == at::kInt, "slot_of mismatch");
  const int64_t M = w.size(0), k = w.size(1), H = eo.size(1);
  const int32_t* rp = nullptr;
  if (range.has_value()) {
    TORCH_CHECK(range->scalar_type() == at::kInt && range->numel() == 2 && range->is_contiguous(),
                "range must be contiguous int32[2]");
    rp = range->data_ptr<int32_t>();
  }
  at::Tensor y = out.has_value() ? as2d(*out) : at::empty({M, H}, eo.options());
  TORCH_CHECK(y.is_contiguous() && y.size(0) == M && y.size(1) == H, "out mismatch");
  launch_moe_combine(eo.data_ptr(), slot_of.data_ptr<int32_t>(), w.data_ptr<float>(), y.data_ptr(), (int)M, (int)k,
                     (int)H, rp, cur_stream());
  return y;
}

at::Tensor grouped_gemm(const at::Tensor& X, const at::Tensor& offsets, const at::Tensor& W, int64_t act) {
  check_bf16(X, "X");
  check_bf16(W, "W");
  TORCH_CHECK(X.dim() == 2 && X.is_contiguous(), "X must be contiguous [rows][K]");
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous(), "W must be contiguous [E][N][K]");
  TORCH_CHECK(offsets.scalar_type() == at::kInt && offsets.numel() == W.size(0) + 1, "offsets must be int32 [E+1]");
  const int64_t rows = X.size(0), K = X.size(1), E = W.size(0), N = W.size(1);
  TORCH_CHECK(W.size(2) == K && K % 8 == 0, "W must be [E][N][K]");
  auto Y = at::empty({rows, N}, X.options());
  if (rows == 0) return Y;
  launch_grouped_gemm(X.data_ptr(), offsets.data_ptr<int32_t>(), W.data_ptr(), Y.data_ptr(), (int)E, (int)N, (int)K,
                      (int)rows, (int)act, cur_stream());
  return Y;
}

// Every expert of an MoE layer in ONE LDS-DMA GEMM launch. x: expert-sorted rows [R][K];
// weights: E tensors [N][K] (validated here) whose addresses the caller caches in w_ptrs
// (int64 [E] on the device: hipGraph-safe); offsets int32 [E+1]. Output: `out` [R][N'] at the
// rows' own positions, or (outs + out_ptrs) E compact outputs, rows 0..min(count, cap)-1 each.
void gemm_grouped(const at::Tensor& x, const std::vector<at::Tensor>& weights, const at::Tensor& w_ptrs,
                  const at::Tensor& offsets, int64_t act, const c10::optional<at::Tensor>& out,
                  const std::vector<at::Tensor>& outs, const c10::optional<at::Tensor>& out_ptrs, int64_t config,
                  const c10::optional<at::Tensor>& a_rows, bool shared_weights) {
  const int64_t E = (int64_t)weights.size();
  check_bf16(x, "x");
  check_rows(x, "x");
  TORCH_CHECK(E > 0, "at least one expert");
  // a_rows (int32 [R], values < x.size(0)): x is the token matrix and sorted row r reads token
  // a_rows[r] (the MoE permute folded into the GEMM's DMA source addresses)
  const int* arp = nullptr;
  if (a_rows.has_value()) {
    TORCH_CHECK(a_rows->is_cuda() && a_rows->scalar_type() == at::kInt && a_rows->is_contiguous(),
                "a_rows: contiguous int32 on the GPU");
    arp = a_rows->data_ptr<int32_t>();
  }
  const int64_t R = a_rows.has_value() ? a_rows->numel() : x.size(0), K = x.size(1), N = weights[0].size(0);
  const bool sw = act == kActSwiglu;
  const int64_t NO = sw ? N / 2 : N;
  for (const auto& w : weights) {
    check_bf16(w, "expert weight");
    TORCH_CHECK(w.is_contiguous() && w.dim() == 2 && w.size(0) == N && w.size(1) == K, "expert weights [N][K]");
  }
  TORCH_CHECK(w_ptrs.is_cuda() && w_ptrs.scalar_type() == at::kLong && w_ptrs.numel() == E, "w_ptrs int64 [E]");
  TORCH_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.numel() == E + 1,
              "offsets int32 [E+1]");
  const int cfg = (int)(config < 0 ? 3 : config);
  TORCH_CHECK((cfg & (kGemmPersist - 1)) < gemm_glds_num_configs() && K % gemm_glds_kstep(cfg) == 0,
              "grouped GEMM: config ", cfg, " needs K % ", gemm_glds_kstep(cfg), " == 0");
  TORCH_CHECK(!sw || N % 32 == 0, "SwiGLU needs interleaved gate/up rows (N % 32 == 0)");
  GemmArgs g{};
  g.A = x.data_ptr();
  g.lda = (int)x.stride(0);
  g.ldw = (int)K;
  g.M = (int)R;
  g.N = (int)N;
  g.K = (int)K;
  g.act = (int)act;
  g.alpha = 1.0f;
  g.grouped_shared = shared_weights ? 1 : 0;
  const unsigned long long* cp = nullptr;
  if (out_ptrs.has_value()) {
    TORCH_CHECK((int64_t)outs.size() == E && out_ptrs->is_cuda() && out_ptrs->scalar_type() == at::kLong &&
                    out_ptrs->numel() == E,
                "compact outputs: E tensors + int64 [E] addresses");
    const int64_t cap = outs[0].size(0);
    for (const auto& o : outs) {
      check_bf16(o, "expert output");
      TORCH_CHECK(o.dim() == 2 && o.is_contiguous() && o.size(1) == NO && o.size(0) == cap,
                  "expert outputs: E contiguous [cap][N'] tensors");
    }
    g.ldc = (int)NO;
    g.compact_rows = (int)cap;
    cp = reinterpret_cast<const unsigned long long*>(out_ptrs->data_ptr<int64_t>());
  } else {
    TORCH_CHECK(out.has_value(), "grouped GEMM needs `out` or compact outputs");
    check_bf16(*out, "out");
    check_rows(*out, "out");
    TORCH_CHECK(out->size(0) == R && out->size(1) == NO, "out must be [R][N'] (N' = N/2 with SwiGLU)");
    g.C = out->data_ptr();
    g.ldc = (int)out->stride(0);
  }
  launch_gemm_glds_grouped(g, cfg, (int)E, offsets.data_ptr<int32_t>(),
                           reinterpret_cast<const unsigned long long*>(w_ptrs.data_ptr<int64_t>()), cp, cur_stream(),
                           arp);
}

// experts: list of E compact [rows][H] bf16 outputs; ptrs: int64 [E] device tensor holding
// their addresses (built once by the caller and cached — hipGraph-safe)
at::Tensor moe_gather_combine(const std::vector<at::Tensor>& experts, const at::Tensor& ptrs, const at::Tensor& idx,
                              const at::Tensor& slot_of, const at::Tensor& offsets, const at::Tensor& w,
                              const c10::optional<at::Tensor>& residual, at::Tensor& out,
                              const c10::optional<at::Tensor>& norm_out, const c10::optional<at::Tensor>& norm_w,
                              const c10::optional<at::Tensor>& norm_b, int64_t norm_mode, double norm_eps) {
  const int64_t E = (int64_t)experts.size();
  TORCH_CHECK(E > 0 && ptrs.scalar_type() == at::kLong && ptrs.numel() == E && ptrs.is_cuda(), "ptrs: int64 [E]");
  const int64_t M = out.size(0), H = out.size(1), k = idx.size(1);
  check_bf16(out, "out");
  TORCH_CHECK(out.is_contiguous() && H % 8 == 0 && k <= 8, "out contiguous [M][H], H % 8 == 0, top-k <= 8");
  for (const auto& t : experts) {
    check_bf16(t, "expert output");
    TORCH_CHECK(t.is_contiguous() && t.size(-1) == H && t.numel() >= M * H, "expert outputs must be [>=M][H]");
  }
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.numel() == M * k && slot_of.scalar_type() == at::kInt &&
                  slot_of.numel() == M * k && offsets.scalar_type() == at::kInt && offsets.numel() == E + 1 &&
                  w.scalar_type() == at::kFloat && w.numel() == M * k,
              "routing tensors: idx/slot int32 [M][k], offsets int32 [E+1], w fp32 [M][k]");
  const void* rp = nullptr;
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->is_contiguous() && residual->numel() == M * H, "residual [M][H]");
    rp = residual->data_ptr();
  }
  void* yn = nullptr;
  const void *nwp = nullptr, *nbp = nullptr;
  if (norm_out.has_value()) {  // post-norm of the combined rows for the next norm
    TORCH_CHECK(norm_mode == 1 || norm_mode == 2, "norm_mode: 1 LayerNorm, 2 RMSNorm");
    TORCH_CHECK(H <= 8192, "post-norm rows hold at most 8192 columns");
    check_bf16(*norm_out, "norm_out");
    check_bf16(*norm_w, "norm_w");
    TORCH_CHECK(norm_out->is_contiguous() && norm_out->numel() == M * H && norm_w.has_value() &&
                    norm_w->is_contiguous() && norm_w->numel() == H,
                "norm_out contiguous [M][H], norm_w [H]");
    TORCH_CHECK(norm_mode == 2 || (norm_b.has_value() && norm_b->is_contiguous() && norm_b->numel() == H),
                "LayerNorm post-norm needs norm_b [H]");
    yn = norm_out->data_ptr();
    nwp = norm_w->data_ptr();
    nbp = norm_mode == 1 ? norm_b->data_ptr() : nullptr;
  } else {
    TORCH_CHECK(H <= 8192, "gather-combine rows hold at most 8192 columns");
  }
  launch_moe_gather_combine(reinterpret_cast<const unsigned long long*>(ptrs.data_ptr<int64_t>()),
                            idx.data_ptr<int32_t>(), slot_of.data_ptr<int32_t>(), offsets.data_ptr<int32_t>(),
                            w.data_ptr<float>(), rp, out.data_ptr(), (int)M, (int)k, (int)H, (int)E, cur_stream(), yn,
                            nwp, nbp, (int)norm_mode, (float)norm_eps);
  return out;
}

}  // namespace

// dst[:src.numel()] <- src: a pinned host uint8 tensor pulled into a GPU uint8 tensor by a kernel
void host_pull(const at::Tensor& dst, const at::Tensor& src, int64_t blocks) {
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous() && dst.scalar_type() == at::kByte, "dst: contiguous GPU uint8");
  TORCH_CHECK(!src.is_cuda() && src.is_pinned() && src.is_contiguous() && src.scalar_type() == at::kByte,
              "src: contiguous pinned host uint8");
  const int64_t n = src.numel();
  TORCH_CHECK(dst.numel() >= n && n % 16 == 0, "sizes: dst >= src, multiple of 16 bytes");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "16-byte alignment");
  TORCH_CHECK(blocks >= 1 && blocks <= 4096, "blocks");
  void* dev_src = nullptr;
  TORCH_CHECK(hipHostGetDevicePointer(&dev_src, src.data_ptr(), 0) == hipSuccess && dev_src != nullptr,
              "pinned host image is not mapped into the GPU address space");
  launch_host_pull(dev_src, dst.data_ptr(), n, (int)blocks, cur_stream());
}

// A device buffer with HIP allocation flags (hipDeviceMallocUncached = 3: reads and writes bypass
// the caches, so a once-per-step stream — the LM head's 77 MB weight, its 51 MB of logits —
// does not evict the layer weights from the 256 MB Infinity Cache). Freed with the tensor.
at::Tensor alloc_device(int64_t nbytes, int64_t flags) {
  TORCH_CHECK(nbytes > 0 && (flags == 0 || flags == 1 || flags == 3), "alloc_device: bytes > 0, flags 0/1/3");
  void* p = nullptr;
  TORCH_CHECK(hipExtMallocWithFlags(&p, (size_t)nbytes, (unsigned)flags) == hipSuccess && p, "hipExtMallocWithFlags failed");
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipFree(q); },
                          at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
}

bool attn_block_ok(int64_t M, int64_t H, int64_t B, int64_t S, int64_t n_head, int64_t n_kv_head, int64_t D) {
  return attn_block_supported((int)M, (int)H, (int)B, (int)S, (int)n_head, (int)n_kv_head, (int)D);
}

int64_t attn_block_sync_size(int64_t M, int64_t S, int64_t B, int64_t n_head) {
  return attn_block_sync_ints((int)M, (int)S, (int)B, (int)n_head) + 1;  // + the error word
}

// The one-launch attention block (attn_block.hip). ``sync``: attn_block_sync_size() int32,
// zeroed once (the launch resets its counters; the last element is the error word).
void attn_block(const at::Tensor& x_in, const at::Tensor& w1, const c10::optional<at::Tensor>& b1,
                const at::Tensor& colsum1, const at::Tensor& ext_stats, int64_t ln_mode, double eps,
                const at::Tensor& qkv_in, const at::Tensor& o_in, const at::Tensor& wo,
                const c10::optional<at::Tensor>& bo, const at::Tensor& res_in, const at::Tensor& out_in,
                const c10::optional<at::Tensor>& stats_out, int64_t B, int64_t S, int64_t n_head, double scale,
                const at::Tensor& sync, int64_t spin_limit, const c10::optional<at::Tensor>& stamps) {
  at::Tensor x = as2d(x_in), qkv = as2d(qkv_in), o = as2d(o_in), r = as2d(res_in), out = as2d(out_in);
  for (auto* t : {&x, &qkv, &o, &r, &out}) {
    check_bf16(*t, "attn_block operand");
    check_rows(*t, "attn_block operand");
  }
  check_bf16(w1, "w1");
  check_bf16(wo, "wo");
  check_rows(w1, "w1");
  check_rows(wo, "wo");
  const int64_t M = x.size(0), H = x.size(1);
  TORCH_CHECK(w1.size(0) == 3 * H && w1.size(1) == H && wo.size(0) == H && wo.size(1) == H && qkv.size(0) == M &&
                  qkv.size(1) == 3 * H && o.size(0) == M && o.size(1) == H && r.size(0) == M && r.size(1) == H &&
                  out.size(0) == M && out.size(1) == H,
              "attn_block: x [M][H], w1 [3H][H], qkv [M][3H], o [M][H], wo [H][H], residual / out [M][H]");
  TORCH_CHECK(H % n_head == 0 && attn_block_ok(M, H, B, S, n_head, n_head, H / n_head),
              "attn_block: shape not supported (M ", M, ", H ", H, ", B ", B, ", S ", S, ", heads ", n_head, ")");
  TORCH_CHECK(ln_mode == 1 || ln_mode == 2, "attn_block: ln_mode 1 LayerNorm, 2 RMSNorm");
  auto f32 = [&](const at::Tensor& t, int64_t n, const char* name) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, name,
                " must be a contiguous fp32 GPU tensor of ", n, " elements");
  };
  f32(colsum1, 3 * H, "colsum1");
  f32(ext_stats, 2 * M, "ext_stats");
  if (stats_out.has_value()) f32(*stats_out, 2 * M, "stats_out");
  for (auto* b : {&b1, &bo})
    if (b->has_value()) {
      check_bf16(**b, "bias");
      TORCH_CHECK((*b)->is_contiguous(), "bias must be contiguous");
    }
  TORCH_CHECK(!b1.has_value() || b1->numel() == 3 * H, "b1 must be [3H]");
  TORCH_CHECK(!bo.has_value() || bo->numel() == H, "bo must be [H]");
  const int64_t n_sync = attn_block_sync_size(M, S, B, n_head);
  TORCH_CHECK(sync.is_cuda() && sync.scalar_type() == at::kInt && sync.is_contiguous() && sync.numel() >= n_sync,
              "sync must be a zeroed int32 GPU tensor of >= ", n_sync, " elements");
  AttnBlockArgs p{x.data_ptr(), (int)x.stride(0), w1.data_ptr(), b1.has_value() ? b1->data_ptr() : nullptr,
                  colsum1.data_ptr<float>(), ext_stats.data_ptr<float>(), (int)ln_mode, (float)eps,
                  qkv.data_ptr(), (int)qkv.stride(0), o.data_ptr(), (int)o.stride(0), wo.data_ptr(),
                  bo.has_value() ? bo->data_ptr() : nullptr, r.data_ptr(), (int)r.stride(0), out.data_ptr(),
                  (int)out.stride(0), stats_out.has_value() ? stats_out->data_ptr<float>() : nullptr, (int)M, (int)H,
                  (int)B, (int)S, (int)n_head, (float)scale, sync.data_ptr<int>(),
                  sync.data_ptr<int>() + (n_sync - 1), (int)spin_limit};
  if (stamps.has_value()) {
    TORCH_CHECK(stamps->is_cuda() && stamps->scalar_type() == at::kLong && stamps->is_contiguous(),
                "stamps must be a contiguous int64 GPU tensor");
    p.stamps = reinterpret_cast<unsigned long long*>(stamps->data_ptr<int64_t>());
  }
  launch_attn_block(p, cur_stream());
}

void register_runner(py::module& m);  // runner.cpp
void register_p2p(py::module& m);     // p2p_binding.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "Hand-written HIP/CDNA4 (gfx950) kernels for distributed_llm_scheduler_amd";
  register_runner(m);
  register_p2p(m);
  m.def("attn_block_ok", &attn_block_ok);
  m.def("attn_block_sync_size", &attn_block_sync_size);
  m.def("attn_block", &attn_block, py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("colsum1"),
        py::arg("ext_stats"), py::arg("ln_mode"), py::arg("eps"), py::arg("qkv"), py::arg("o"), py::arg("wo"),
        py::arg("bo"), py::arg("residual"), py::arg("out"), py::arg("stats_out"), py::arg("B"), py::arg("S"),
        py::arg("n_head"), py::arg("scale"), py::arg("sync"), py::arg("spin_limit"),
        py::arg("stamps") = py::none());
  m.def("alloc_device", &alloc_device, py::arg("nbytes"), py::arg("flags") = 3);
  m.def("host_pull", &host_pull, py::arg("dst"), py::arg("src"), py::arg("blocks") = 256);
  m.def("gemm", &gemm, py::arg("a"), py::arg("w"), py::arg("bias") = py::none(), py::arg("residual") = py::none(),
        py::arg("act") = 0, py::arg("alpha") = 1.0, py::arg("out") = py::none(), py::arg("config") = -1,
        py::arg("splitk") = 0, py::arg("ln_colsum") = py::none(), py::arg("ln_mode") = 0, py::arg("ln_eps") = 1e-5,
        py::arg("rows") = py::none(), py::arg("compact_rows") = false, py::arg("rope_cos") = py::none(),
        py::arg("rope_sin") = py::none(), py::arg("rope_S") = 1, py::arg("rope_D") = 2, py::arg("rope_cols") = 0,
        py::arg("stats_out") = py::none(), py::arg("ext_stats") = py::none(), py::arg("norm_out") = py::none(),
        py::arg("norm_w") = py::none(), py::arg("norm_b") = py::none(), py::arg("norm_mode") = 0,
        py::arg("norm_eps") = 1e-5, py::arg("stream_pol") = 0);
  m.attr("REGSTAGE") = kRegStage;
  m.attr("PERSIST") = kGemmPersist;
  m.def("gemm_pick_config", &gemm_pick_config);
  m.def("gemm_glds_num_configs", &gemm_glds_num_configs);
  m.def("gemm_glds_kstep", &gemm_glds_kstep);
  m.def("gemm_glds_pick", [](int M, int N, int K) {
    int c, s;
    gemm_glds_pick(M, N, K, &c, &s);
    return std::make_pair(c, s);
  });
  m.def("attention", &attention, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("B"), py::arg("S"),
        py::arg("n_head"), py::arg("n_kv_head"), py::arg("head_dim"), py::arg("causal") = true,
        py::arg("scale") = 0.125, py::arg("out") = py::none(), py::arg("variant") = 0, py::arg("Sq") = 0,
        py::arg("q_off") = 0, py::arg("flags") = 0);
  m.def("norm", &norm, py::arg("x"), py::arg("w"), py::arg("b") = py::none(), py::arg("eps") = 1e-5,
        py::arg("residual") = py::none(), py::arg("rms") = false, py::arg("out") = py::none(),
        py::arg("sum_out") = py::none());
  m.def("gelu", &gelu, py::arg("x"), py::arg("out") = py::none());
  m.def("add", &add, py::arg("a"), py::arg("b"), py::arg("out") = py::none());
  m.def("swiglu", &swiglu, py::arg("gate_up"), py::arg("out") = py::none());
  m.def("mlp_fused", &mlp_fused);
  m.def("mlp_fused_ok", &mlp_fused_ok);
  m.def("embedding", &embedding, py::arg("tokens"), py::arg("wte"), py::arg("wpe") = py::none(), py::arg("S") = 1,
        py::arg("out") = py::none(), py::arg("zero") = py::none(), py::arg("stats") = py::none());
  m.def("rope_", &rope_);
  m.def("moe_router", &moe_router);
  m.def("moe_gather_combine", &moe_gather_combine, py::arg("experts"), py::arg("ptrs"), py::arg("idx"),
        py::arg("slot_of"), py::arg("offsets"), py::arg("w"), py::arg("residual"), py::arg("out"),
        py::arg("norm_out") = py::none(), py::arg("norm_w") = py::none(), py::arg("norm_b") = py::none(),
        py::arg("norm_mode") = 0, py::arg("norm_eps") = 1e-5);
  m.def("moe_align", &moe_align);
  m.def("moe_route", &moe_route);
  m.def("moe_gate_route", &moe_gate_route);
  m.def("moe_pack", &moe_pack);
  m.def("moe_permute", &moe_permute, py::arg("x"), py::arg("src_rows"), py::arg("out") = py::none());
  m.def("moe_xbatch_index", &moe_xbatch_index);
  m.def("moe_combine", &moe_combine, py::arg("expert_out"), py::arg("slot_of"), py::arg("weights"),
        py::arg("range") = py::none(), py::arg("out") = py::none());
  m.def("grouped_gemm", &grouped_gemm, py::arg("X"), py::arg("offsets"), py::arg("W"), py::arg("act") = 0);
  m.def("gemm_grouped", &gemm_grouped, py::arg("x"), py::arg("weights"), py::arg("w_ptrs"), py::arg("offsets"),
        py::arg("act") = 0, py::arg("out") = py::none(), py::arg("outs") = std::vector<at::Tensor>{},
        py::arg("out_ptrs") = py::none(), py::arg("config") = -1, py::arg("a_rows") = py::none(),
        py::arg("shared_weights") = false);
}
