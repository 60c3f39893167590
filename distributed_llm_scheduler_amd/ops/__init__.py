"""Operator layer: hand-written HIP/CDNA4 kernels with fp32 PyTorch references.

``ops.linear(x, w, ...)`` etc. dispatch on the tensor's device:

* GPU tensors run the HIP kernels in ``_dlsched_ops`` (csrc/kernels/*.hip, built for
  gfx950). If the extension cannot be loaded on a GPU box this raises — there is no
  silent eager fallback for GPU tensors.
* CPU tensors run the ``ref_*`` implementations (fp32 math, result cast back to the
  input dtype). They define the numerics the kernels are tested against and power the
  CPU "fake device" executor used by the multi-process tests.

Weight layout everywhere: GEMM weights are ``[N][K]`` (K contiguous); ``y = x @ W^T``.
"""
from __future__ import annotations

import math
import os
import threading
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import tuning

ACT = {None: 0, "none": 0, "gelu": 1, "gelu_tanh": 1, "silu": 2, "relu": 3, "swiglu": 4}
SWIGLU = 4
SWIGLU_BLOCK = 16  # gate/up interleave granularity of a SwiGLU-epilogue weight (csrc common.h)
# cache policy of vocabulary-sized projections (the LM head: a weight read once per step and a
# write-once logits tensor; GemmArgs::stream_pol): bit 0 weight DMA nt, bit 1 output stores nt.
# Streaming both keeps GPT-2's 170 MB of layer weights resident in the 256 MB Infinity Cache
# from step to step (its 77 MB LM-head weight and 51 MB of logits otherwise push them out):
# step 0.639 vs 0.689 ms (profiles/r4_ab/lmhead_stream_policy.txt)
LMHEAD_POL = int(os.environ.get("DLS_LMHEAD_POL", "3"))
LMHEAD_MIN_N = 32000
# weights of at least this many MB DMA'd with the nt policy (0: off) — for models whose weights
# stream from HBM every step anyway (A/B knob)
WEIGHT_NT_MB = float(os.environ.get("DLS_WEIGHT_NT_MB", "0"))
# cache policy bits of every other GEMM launch: 2 output stores nt, 4 output stores
# write-through (sc1) — bf16 outputs, split-K partial slabs and their reduce kernels' outputs
# leave the XCD's L2 as they are written, so the kernel boundary has no dirty lines to write
# back: GPT-2 0.620 vs 0.640 ms, Llama-3-8B 9.46 vs 9.49 ms (profiles/r4_ab/write_through.txt);
# nt output stores cost GPT-2 5 %
ACT_POL = int(os.environ.get("DLS_ACT_POL", "4"))
# per-model default where the measurement disagrees (DLS_ACT_POL, when set, wins): Mixtral-8x7B's
# step is faster with default-policy output stores, 24.40 / 24.50 vs 24.68 / 24.75 ms
# (profiles/r5_ab/knob_recheck.txt)
ACT_POL_MODEL = {"mixtral-8x7b": 0}
_ACT_POL_SET = "DLS_ACT_POL" in os.environ
# attention flags: bit 0 output stores write-through (no measurable difference), bit 1 the
# blocks of one head grouped on one XCD (A/B knob)
ATTN_FLAGS = int(os.environ.get("DLS_ATTN_FLAGS", "0"))
# attention kernel variant (0: the launcher's choice by grid size; 1..13: attention.hip)
ATTN_VARIANT = int(os.environ.get("DLS_ATTN_VARIANT", "0"))


# the LM-head policy pays only while the model's layer weights can stay MALL-resident: a
# vocabulary projection whose own weight is this large belongs to a model whose weights stream
# from HBM every step anyway, and there nt weight DMA slows the LM head itself (Llama-3-8B's
# 1 GB LM head: 683 vs 432 us per step, profiles/r4_ab/lmhead_stream_policy.txt)
LMHEAD_POL_MAX_MB = 128


def _stream_pol(N: int, K: int) -> int:
    lm = N >= LMHEAD_MIN_N and N * K * 2 <= LMHEAD_POL_MAX_MB * 1e6
    pol = LMHEAD_POL if lm else (ACT_POL if _ACT_POL_SET else ACT_POL_MODEL.get(tuning._model, ACT_POL))
    if WEIGHT_NT_MB > 0 and N * K * 2 >= WEIGHT_NT_MB * 1e6:
        pol |= 1
    return pol

_lock = threading.Lock()
_ext = None
_ext_err: Optional[BaseException] = None


def _load_ext():
    global _ext, _ext_err
    if _ext is not None:
        return _ext
    with _lock:
        if _ext is None:
            try:
                from .. import _build
                if os.environ.get("DLS_SKIP_BUILD") != "1":
                    _build.build_ops()
                import importlib
                _ext = importlib.import_module("distributed_llm_scheduler_amd._dlsched_ops")
            except BaseException as e:  # noqa: BLE001 - re-raised with context in ext()
                _ext_err = e
    return _ext


def ext():
    """The compiled HIP op library; raises if it is unavailable (never falls back)."""
    m = _load_ext()
    if m is None:
        raise RuntimeError(f"HIP kernel library _dlsched_ops is not available: {_ext_err!r}")
    return m


def native_available() -> bool:
    return _load_ext() is not None


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ----------------------------------------------------------------- references (fp32)

def _act_ref(y: torch.Tensor, act) -> torch.Tensor:
    a = ACT[act] if not isinstance(act, int) else act
    if a == 1:
        return F.gelu(y, approximate="tanh")
    if a == 2:
        return F.silu(y)
    if a == 3:
        return F.relu(y)
    return y


def interleave_gate_up(w: torch.Tensor) -> torch.Tensor:
    """[gate (F rows); up (F rows)] -> rows interleaved in blocks of 16 (gate 16c..16c+15, then
    up 16c..16c+15) — the layout the GEMM's SwiGLU epilogue pairs fragments in. Works for a
    weight [2F, K] or a per-row vector [2F] (bias, colsum)."""
    F2 = w.shape[0]
    assert F2 % (2 * SWIGLU_BLOCK) == 0, "SwiGLU width must be a multiple of 16"
    F = F2 // 2
    rest = tuple(w.shape[1:])
    g = w[:F].reshape((F // SWIGLU_BLOCK, SWIGLU_BLOCK) + rest)
    u = w[F:].reshape((F // SWIGLU_BLOCK, SWIGLU_BLOCK) + rest)
    return torch.stack([g, u], 1).reshape((F2,) + rest).contiguous()


def rope_pair_perm(n_q_heads: int, n_k_heads: int, head_dim: int, total_rows: int) -> torch.Tensor:
    """Row order making every RoPE pair adjacent within each q / k head: new row 2i of a head
    is its old row i, new 2i+1 is old i + D/2 (V rows untouched). q.k is invariant under a
    permutation applied to both, so attention needs nothing else."""
    half = head_dim // 2
    within = torch.stack([torch.arange(half), torch.arange(half) + half], 1).reshape(-1)
    idx = torch.arange(total_rows)
    for h in range(n_q_heads + n_k_heads):
        idx[h * head_dim:(h + 1) * head_dim] = h * head_dim + within
    return idx


def _rope_ref_pairs(y: torch.Tensor, rope) -> torch.Tensor:
    cos_t, sin_t, S, D, cols = rope
    M = y.shape[0]
    pos = torch.arange(M) % S
    c = cos_t.cpu()[pos].float()
    sn = sin_t.cpu()[pos].float()
    heads = cols // D
    v = y[:, :cols].reshape(M, heads, D // 2, 2)
    x0, x1 = v[..., 0], v[..., 1]
    cc, ss = c[:, None, :], sn[:, None, :]
    out = torch.stack([x0 * cc - x1 * ss, x1 * cc + x0 * ss], -1).reshape(M, cols)
    return torch.cat([out, y[:, cols:]], 1)


def _swiglu_interleaved(y: torch.Tensor) -> torch.Tensor:
    F2 = y.shape[-1]
    v = y.reshape(y.shape[:-1] + (F2 // (2 * SWIGLU_BLOCK), 2, SWIGLU_BLOCK))
    return (F.silu(v[..., 0, :]) * v[..., 1, :]).reshape(y.shape[:-1] + (F2 // 2,))


def ref_linear(x, w, bias=None, act=None, residual=None, alpha=1.0, rope=None):
    y = alpha * (x.float() @ w.float().t())
    if bias is not None:
        y = y + bias.float()
    if rope is not None:
        y = _rope_ref_pairs(y.reshape(-1, y.shape[-1]), rope).reshape(y.shape)
    if (ACT[act] if not isinstance(act, int) else act) == SWIGLU:
        y = _swiglu_interleaved(y)
        return (y if residual is None else y + residual.float()).to(x.dtype)
    y = _act_ref(y, act)
    if residual is not None:
        y = y + residual.float()
    return y.to(x.dtype)


def ref_layernorm(x, w, b, eps=1e-5):
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), None if b is None else b.float(), eps).to(x.dtype)


def ref_rmsnorm(x, w, eps=1e-5):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


def ref_attention(q, k, v, B, S, n_head, n_kv_head, head_dim, causal=True, scale=None, Sq=None, q_off=0):
    """q [B*Sq][>=nh*D], k/v [B*S][>=nkv*D] (row views into a packed qkv buffer allowed).
    ``Sq``/``q_off``: the queries are the sequence chunk at positions q_off .. q_off+Sq-1
    attending keys 0 .. S-1 (causal: key <= query position)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    Sq = S if Sq is None else Sq
    qh = q[:, :n_head * head_dim].float().reshape(B, Sq, n_head, head_dim).transpose(1, 2)
    kh = k[:, :n_kv_head * head_dim].float().reshape(B, S, n_kv_head, head_dim).transpose(1, 2)
    vh = v[:, :n_kv_head * head_dim].float().reshape(B, S, n_kv_head, head_dim).transpose(1, 2)
    rep = n_head // n_kv_head
    if rep > 1:
        kh = kh.repeat_interleave(rep, dim=1)
        vh = vh.repeat_interleave(rep, dim=1)
    s = (qh @ kh.transpose(-1, -2)) * scale
    if causal:
        qpos = torch.arange(Sq, device=q.device)[:, None] + q_off
        mask = torch.arange(S, device=q.device)[None, :] > qpos
        s = s.masked_fill(mask, float("-inf"))
    o = torch.softmax(s, dim=-1) @ vh
    return o.transpose(1, 2).reshape(B * Sq, n_head * head_dim).to(q.dtype)


def rope_tables(S: int, head_dim: int, theta: float, device="cpu") -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None, :]
    return ang.cos().float().contiguous().to(device), ang.sin().float().contiguous().to(device)


def ref_rope_(qkv, S, n_head, n_kv_head, head_dim, k_col, cos_t, sin_t):
    M = qkv.shape[0]
    pos = torch.arange(M, device=qkv.device) % S
    c, s = cos_t[pos].to(qkv.device), sin_t[pos].to(qkv.device)
    half = head_dim // 2

    def rot(view, heads):
        x = view.float().reshape(M, heads, head_dim)
        x1, x2 = x[..., :half], x[..., half:]
        cc, ss = c[:, None, :], s[:, None, :]
        out = torch.cat([x1 * cc - x2 * ss, x2 * cc + x1 * ss], dim=-1)
        view.copy_(out.reshape(M, heads * head_dim).to(view.dtype))

    rot(qkv[:, :n_head * head_dim], n_head)
    rot(qkv[:, k_col:k_col + n_kv_head * head_dim], n_kv_head)
    return qkv


# --------------------------------------------------------------------- dispatchers

def _post_norm_args(post_norm):
    """(out, w, b, kind, eps) -> kwargs of the native post-norm (kind "layernorm" / "rmsnorm")."""
    y, nw, nb, kind, eps = post_norm
    return dict(norm_out=y, norm_w=nw, norm_b=nb if kind == "layernorm" else None,
                norm_mode=1 if kind == "layernorm" else 2, norm_eps=float(eps))


def _post_norm_ref(src, post_norm):
    y, nw, nb, kind, eps = post_norm
    s2 = src.reshape(-1, src.shape[-1])
    r = ref_layernorm(s2, nw, nb, eps) if kind == "layernorm" else ref_rmsnorm(s2, nw, eps)
    y.view(r.shape).copy_(r)


def linear(x, w, bias=None, act=None, residual=None, alpha=1.0, out=None, rows=None, rows_hint=None,
           compact=False, rope=None, stats_out=None, post_norm=None):
    """``act(alpha * x @ w^T + bias) + residual`` — one MFMA GEMM kernel with the whole
    epilogue fused on GPU. ``act="swiglu"`` takes a gate/up-interleaved weight
    (:func:`interleave_gate_up`) and returns the N/2-wide ``silu(gate) * up``. ``rows``
    (int32[2] tensor on x's device) restricts the GEMM to rows [rows[0], rows[1]) of x and
    ``out`` without a host sync (MoE experts); ``rows_hint`` is the expected row count used
    to pick the tuned kernel config; ``compact`` writes the range to rows 0..r1-r0-1 of ``out``
    (at most ``out.shape[0]`` rows). ``rope=(cos, sin, S, D, cols)`` rotates output columns
    [0, cols) in the epilogue (q/k rows pair-interleaved, :func:`rope_pair_perm`). ``stats_out``
    (GPU, fp32 [M, 2], zeroed by the caller): accumulate each output row's (sum, sum of
    squares) for the next folded norm (:func:`linear_norm` ``ext_stats``). ``post_norm =
    (y, w, b, "rmsnorm" | "layernorm", eps)``: also write the NEXT norm of the output rows into
    ``y`` (a split-K launch does it in its row-owning reduce, saving the norm launch)."""
    a = ACT[act] if not isinstance(act, int) else act
    n_out = w.shape[0] // 2 if a == SWIGLU else w.shape[0]
    if _gpu(x):
        shp = x.shape[:-1] + (n_out,)
        M = x.numel() // x.shape[-1]
        cfg, sk = tuning.lookup(rows_hint or M, w.shape[0], w.shape[1], tuning.tag(a, rows is not None))
        if cfg == tuning.LIB:  # (only with DLS_ALLOW_VENDOR_GEMM=1: tuning.lookup)
            if tuning.VENDOR and a == 0 and residual is None and rows is None and rope is None \
                    and stats_out is None and post_norm is None:
                # opt-in: a PLAIN GEMM (no fused epilogue) whose tuned choice is the vendor
                # library (hipBLASLt via torch); every fused-epilogue GEMM stays on the HIP kernels
                x2 = x.reshape(M, x.shape[-1])
                o2 = out.view(M, n_out) if out is not None else torch.empty(M, n_out, dtype=x.dtype, device=x.device)
                if bias is not None:
                    torch.addmm(bias, x2, w.t(), beta=1.0, alpha=float(alpha), out=o2)
                else:
                    torch.mm(x2, w.t(), out=o2)
                    if alpha != 1.0:
                        o2.mul_(alpha)
                return o2.view(shp) if out is None else out
            cfg, sk = tuning.lookup_fused(rows_hint or M, w.shape[0], w.shape[1], tuning.tag(a, rows is not None))
        rc, rs_, rS, rD, rcols = rope if rope is not None else (None, None, 1, 2, 0)
        y = ext().gemm(x, w, bias, residual, a, float(alpha), out, cfg, sk, None, 0, 1e-5, rows, bool(compact),
                       rc, rs_, int(rS), int(rD), int(rcols), stats_out, None,
                       stream_pol=_stream_pol(w.shape[0], w.shape[1]) if rows is None else 0,
                       **(_post_norm_args(post_norm) if post_norm is not None else {}))
        return y.view(shp) if out is None else out
    if rows is not None:
        r0, r1 = (int(v) for v in rows.tolist())
        if out is None:
            out = torch.zeros(x.shape[:-1] + (n_out,), dtype=x.dtype)
        res = residual[r0:r1] if residual is not None else None
        o2 = out.reshape(-1, out.shape[-1])
        if compact:
            n = min(r1 - r0, o2.shape[0])
            o2[:n] = ref_linear(x[r0:r0 + n], w, bias, act, None, alpha)
        else:
            o2[r0:r1] = ref_linear(x[r0:r1], w, bias, act, res, alpha)
        return out
    y = ref_linear(x, w, bias, act, residual, alpha, rope=rope)
    if out is not None:
        out.copy_(y)
        y = out
    if post_norm is not None:
        _post_norm_ref(y, post_norm)
    return y


def derive_norm_gemm(w, ln_w, ln_b=None, bias=None):
    """Fold a norm's affine into the following GEMM: returns (W' = W * ln_w, colsum(W') in
    fp32, bias' = bias + W @ ln_b). W' is rounded to bf16 BEFORE the column sums, so the
    epilogue's mean correction matches exactly what the MFMAs multiply."""
    wf = w.float()
    wd = (wf * ln_w.float()[None, :]).to(w.dtype)
    cs = wd.float().sum(1).contiguous()
    b = torch.zeros(w.shape[0], device=w.device) if bias is None else bias.float()
    if ln_b is not None:
        # an elementwise product + row sum, NOT ``wf @ ln_b``: that GEMV would run in the vendor
        # BLAS (hipBLASLt), which EXITS the process (status 1, "operation not permitted when
        # stream is capturing") when first used while another rank thread of the single-GPU
        # harness is capturing a graph — the round-5 driver GPU suite's silent death
        b = b + (wf * ln_b.float()[None, :]).sum(1)
    return wd, cs, b.to(w.dtype).contiguous()


def linear_norm(x, w_derived, colsum, bias_derived, mode, eps=1e-5, act=None, residual=None, out=None, rope=None,
                ext_stats=None):
    """``act(W . norm(x) + bias) + residual`` in ONE GEMM on the raw rows ``x`` (GPU), with
    ``(w_derived, colsum, bias_derived)`` from :func:`derive_norm_gemm`. ``mode`` is
    "layernorm" or "rmsnorm". Row statistics are accumulated in the GEMM's main loop, or —
    with ``ext_stats`` (fp32 [M, 2] sums emitted by x's producer) — read from there, which
    frees the tile config and split-K choice."""
    m = {"layernorm": 1, "rmsnorm": 2}[mode]
    a = ACT[act] if not isinstance(act, int) else act
    shp = x.shape[:-1] + (w_derived.shape[0] // 2 if a == SWIGLU else w_derived.shape[0],)
    M, N, K = x.numel() // x.shape[-1], w_derived.shape[0], w_derived.shape[1]
    split = tuning.col_split(M, N, K, tuning.tag(a)) if ext_stats is not None and rope is None and a != SWIGLU \
        else None
    if split:
        # one launch per column range (e.g. the LM head: a whole round of 256 x 256 tiles, then
        # the remaining columns as one round of 256 x 144 tiles) into column views of ``out``
        if out is None:
            out = torch.empty(shp, dtype=x.dtype, device=x.device)
        o2 = out.view(M, N)
        r2 = residual.reshape(M, N) if residual is not None else None
        pol = _stream_pol(N, K)
        for n0, n1, c, k in split:
            ext().gemm(x, w_derived[n0:n1], bias_derived[n0:n1] if bias_derived is not None else None,
                       r2[:, n0:n1] if r2 is not None else None, a, 1.0, o2[:, n0:n1], int(c), int(k),
                       colsum[n0:n1], m, float(eps), None, False, None, None, 1, 2, 0, None, ext_stats,
                       stream_pol=pol)
        return out
    cfg, sk = tuning.lookup_fused(M, N, K, tuning.tag(a))
    if ext_stats is None:
        sk = 1
        if 0 <= cfg < tuning.REGSTAGE and tuning.kstep(cfg) != 64:
            # in-loop row statistics need one K group: the fastest such candidate of the shape
            # instead of the kernel's generic 64x64 fallback
            cfg = next((int(c) for c, _ in tuning.runner_ups(M, N, K, tuning.tag(a), 8)
                        if 0 <= c < tuning.REGSTAGE and tuning.kstep(c) == 64), -1)
    rc, rs_, rS, rD, rcols = rope if rope is not None else (None, None, 1, 2, 0)
    pol = _stream_pol(N, K)
    y = ext().gemm(x, w_derived, bias_derived, residual, a, 1.0, out, cfg if cfg < tuning.REGSTAGE else -1, sk, colsum,
                   m, float(eps), None, False, rc, rs_, int(rS), int(rD), int(rcols), None, ext_stats,
                   stream_pol=pol)
    return y.view(shp) if out is None else out


def mlp_fused_ok(M, H, F, Hout) -> bool:
    """Does the one-launch MLP block (gemm_fused.hip) take this shape on this GPU?"""
    return bool(ext().mlp_fused_ok(int(M), int(H), int(F), int(Hout)))


def mlp_fused(x, w1_derived, b1_derived, colsum1, ext_stats, mode, eps, h, w2, b2, residual, out, stats_out=None,
              sync=None, spin_limit=1 << 22):
    """A pre-norm transformer MLP block as ONE launch (GPU): ``h = GELU(W1'.norm(x) + b1')``
    (norm folded as in :func:`linear_norm`, row statistics handed over in ``ext_stats``) and
    ``out = h W2^T + b2 + residual`` (+ each output row's statistics into ``stats_out``), the two
    GEMMs linked inside the launch (fc1 tiles publish write-through, fc2 tiles start when their
    rows' fc1 tiles have arrived). ``sync``: zeroed int32 [2 * M / 64 + 1]; its last word is set
    if a wait gave up (never expected). ``h`` is written too (it is the DAG's activation)."""
    m = {"layernorm": 1, "rmsnorm": 2}[mode]
    if sync is None:
        sync = torch.zeros(2 * (x.numel() // x.shape[-1]) // 64 + 1, dtype=torch.int32, device=x.device)
    ext().mlp_fused(x, w1_derived, b1_derived, colsum1, ext_stats, m, float(eps), ACT["gelu"], h, w2, b2, residual,
                    out, stats_out, sync, int(spin_limit))
    return out


def attn_block_ok(M, H, B, S, n_head, n_kv_head, head_dim) -> bool:
    """Does the one-launch attention block (attn_block.hip) take this shape?"""
    return bool(ext().attn_block_ok(int(M), int(H), int(B), int(S), int(n_head), int(n_kv_head), int(head_dim)))


def attn_block_sync(M, S, B, n_head, device) -> torch.Tensor:
    """A zeroed counter buffer for :func:`attn_block` (the launch resets it; last word: error)."""
    return torch.zeros(int(ext().attn_block_sync_size(int(M), int(S), int(B), int(n_head))), dtype=torch.int32,
                       device=device)


def attn_block(x, w_qkv_derived, b_qkv_derived, colsum, ext_stats, mode, eps, qkv, o, w_o, b_o, residual, out,
               B, S, n_head, stats_out=None, sync=None, scale=None, spin_limit=1 << 22):
    """A pre-norm attention block as ONE launch (GPU, attn_block.hip): ``qkv = W'.norm(x) + b'``
    (norm folded as in :func:`linear_norm`, row statistics of x in ``ext_stats``), causal MHA
    over ``qkv`` into ``o``, ``out = o W_o^T + b_o + residual`` (+ each output row's statistics
    into ``stats_out``) — the three stages linked inside the launch by per-row-block arrival
    counters (a query tile starts once the q / k / v tiles of its rows and earlier ones exist;
    an out-proj tile once every head of its rows is done). ``qkv`` and ``o`` are written too."""
    m = {"layernorm": 1, "rmsnorm": 2}[mode]
    H = x.shape[-1]
    if sync is None:
        sync = attn_block_sync(x.numel() // H, S, B, n_head, x.device)
    scale = scale if scale is not None else 1.0 / math.sqrt(H // n_head)
    ext().attn_block(x, w_qkv_derived, b_qkv_derived, colsum, ext_stats, m, float(eps), qkv, o, w_o, b_o, residual,
                     out, stats_out, int(B), int(S), int(n_head), float(scale), sync, int(spin_limit))
    return out


def layernorm(x, w, b, eps=1e-5, residual=None, out=None, sum_out=None):
    """LayerNorm; with ``residual`` returns ``(LN(x + residual), x + residual)``."""
    if _gpu(x):
        y, s = ext().norm(x, w, b, float(eps), residual, False, out, sum_out)
        y = y.view(x.shape)
        return (y, s.view(x.shape)) if residual is not None else y
    if residual is not None:
        s = (x.float() + residual.float()).to(x.dtype)
        y = ref_layernorm(s, w, b, eps)
        if sum_out is not None:
            sum_out.copy_(s)
        if out is not None:
            out.copy_(y)
        return y, s
    y = ref_layernorm(x, w, b, eps)
    if out is not None:
        out.copy_(y)
    return y


def rmsnorm(x, w, eps=1e-5, residual=None, out=None, sum_out=None):
    if _gpu(x):
        y, s = ext().norm(x, w, None, float(eps), residual, True, out, sum_out)
        y = y.view(x.shape)
        return (y, s.view(x.shape)) if residual is not None else y
    if residual is not None:
        s = (x.float() + residual.float()).to(x.dtype)
        y = ref_rmsnorm(s, w, eps)
        if sum_out is not None:
            sum_out.copy_(s)
        if out is not None:
            out.copy_(y)
        return y, s
    y = ref_rmsnorm(x, w, eps)
    return out.copy_(y) if out is not None else y


def attention(q, k, v, B, S, n_head, n_kv_head, head_dim, causal=True, scale=None, out=None, Sq=None, q_off=0):
    """Flash attention (GPU) / fp32 reference (CPU). ``Sq``/``q_off``: a sequence chunk of
    queries at positions q_off.. against S keys (sequence-parallel attention nodes)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(head_dim)
    if _gpu(q):
        return ext().attention(q, k, v, B, S, n_head, n_kv_head, head_dim, causal, float(scale), out, ATTN_VARIANT,
                               int(Sq or 0), int(q_off), int(ATTN_FLAGS))
    y = ref_attention(q, k, v, B, S, n_head, n_kv_head, head_dim, causal, scale, Sq=Sq, q_off=q_off)
    if out is not None:
        out.copy_(y)
        return out
    return y


def gelu(x, out=None):
    if _gpu(x):
        return ext().gelu(x.contiguous(), out)
    y = F.gelu(x.float(), approximate="tanh").to(x.dtype)
    return out.copy_(y) if out is not None else y


def add(a, b, out=None):
    if _gpu(a):
        return ext().add(a.contiguous(), b.contiguous(), out)
    y = (a.float() + b.float()).to(a.dtype)
    return out.copy_(y) if out is not None else y


def swiglu(gate_up, out=None):
    if _gpu(gate_up):
        y = ext().swiglu(gate_up, out)
        return y.view(gate_up.shape[:-1] + (gate_up.shape[-1] // 2,))
    f = gate_up.shape[-1] // 2
    y = (F.silu(gate_up[..., :f].float()) * gate_up[..., f:].float()).to(gate_up.dtype)
    return out.copy_(y) if out is not None else y


def embedding(tokens, wte, wpe=None, S=1, out=None, zero=None, stats=None):
    """``wte[tokens] (+ wpe[pos % S])``; ``zero`` (GPU fp32) is cleared by the same kernel;
    ``stats`` (fp32 [rows, 2], disjoint from ``zero``) receives each output row's (sum, sum of
    squares) for the next folded norm."""
    if _gpu(wte):
        return ext().embedding(tokens.to(torch.int32).contiguous(), wte, wpe, int(S), out, zero, stats)
    if zero is not None:
        zero.zero_()
    t = tokens.reshape(-1).long()
    y = wte.float()[t]
    if wpe is not None:
        y = y + wpe.float()[torch.arange(t.numel()) % S]
    y = y.to(wte.dtype)
    if stats is not None:
        yf = y.float()
        stats.view(-1, 2).copy_(torch.stack([yf.sum(1), (yf * yf).sum(1)], 1))
    return out.copy_(y) if out is not None else y


def rope_(qkv, S, n_head, n_kv_head, head_dim, k_col, cos_t, sin_t):
    if _gpu(qkv):
        ext().rope_(qkv, S, n_head, n_kv_head, head_dim, k_col, cos_t, sin_t)
        return qkv
    return ref_rope_(qkv, S, n_head, n_kv_head, head_dim, k_col, cos_t, sin_t)


# ------------------------------------------------------------------------- MoE

def moe_router(logits, topk):
    if _gpu(logits):
        return tuple(ext().moe_router(logits.contiguous(), int(topk)))
    lf = logits.float()
    val, idx = torch.topk(lf, topk, dim=-1)
    w = torch.softmax(val, dim=-1)
    return idx.to(torch.int32), w


def moe_align(topk_idx, n_experts):
    """Counting sort of (token, k) assignments by expert -> (src_rows, slot_of, offsets)."""
    if _gpu(topk_idx):
        return tuple(ext().moe_align(topk_idx.contiguous(), int(n_experts)))
    flat = topk_idx.reshape(-1).long()
    k = topk_idx.shape[1]
    order = torch.sort(flat, stable=True).indices
    slot_of = torch.empty_like(order)
    slot_of[order] = torch.arange(order.numel())
    counts = torch.bincount(flat, minlength=n_experts)
    offsets = torch.zeros(n_experts + 1, dtype=torch.int64)
    offsets[1:] = torch.cumsum(counts, 0)
    return (order // k).to(torch.int32), slot_of.to(torch.int32), offsets.to(torch.int32)


def moe_route(logits, topk, n_experts):
    """Router + align of one MoE layer: (idx, gate, src_rows, slot_of, offsets). GPU: ONE
    workgroup launch (route_kernel) with exactly the outputs of moe_router + moe_align."""
    if _gpu(logits) and logits.shape[0] * topk <= 16384 and logits.shape[1] == n_experts:
        return tuple(ext().moe_route(logits.contiguous(), int(topk)))
    idx, gate = moe_router(logits, topk)
    return (idx, gate) + moe_align(idx, n_experts)


def moe_gate_route(x, w_gate, topk, logits):
    """Router GEMM + routing of one MoE layer: ``logits`` (bf16 [M][E]) <- x @ w_gate^T and
    returns (idx, gate, src_rows, slot_of, offsets). GPU: ONE launch (the last workgroup to
    publish its logits routes every token) when the shape fits the kernel, else the GEMM and
    moe_route."""
    if _gpu(x):
        r = ext().moe_gate_route(x, w_gate, int(topk), logits.view(x.shape[0], -1))
        if r:
            return tuple(r)
    linear(x, w_gate, out=logits.view(x.shape[0], -1))
    return moe_route(logits.view(x.shape[0], -1), topk, w_gate.shape[0])


def moe_permute(x, src_rows, out=None):
    if _gpu(x):
        return ext().moe_permute(x.contiguous(), src_rows, out)
    y = x[src_rows.long()]
    return out.copy_(y) if out is not None else y


def moe_pack(x, src_rows, offsets, dests, ovf, unpack=False):
    """Expert-parallel capacity edges (fixed-size messages; kernels.h MoePackArgs). ``dests``:
    [(buf [cap][H], cap, experts, flag, ecaps, eflags)], one per expert GPU. Pack (``unpack``
    False): buf row c <- token row ``x[src_rows[j]]`` for the c-th routed row of the listed
    experts (expert-sorted order, experts in the listed order). Unpack: ``x`` holds the
    expert-sorted rows and row j <- buf row c. Rows past ``cap`` are not moved and set
    ``ovf[flag]``; an expert whose own count exceeds ``ecaps[k]`` sets ``ovf[eflags[k]]`` (its
    compact output travels back in an edge of that many rows). No host sync on the GPU."""
    if _gpu(x):
        ext().moe_pack(x, src_rows, offsets, [d[0] for d in dests], [int(d[1]) for d in dests],
                       [list(map(int, d[2])) for d in dests], [int(d[3]) for d in dests],
                       [list(map(int, d[4])) for d in dests], [list(map(int, d[5])) for d in dests], ovf, bool(unpack))
        return
    off = [int(v) for v in offsets.tolist()]
    H = x.shape[-1]
    for buf, cap, experts, flag, ecaps, eflags in dests:
        b2 = buf.view(-1)[:int(cap) * H].view(int(cap), H)
        c = 0
        for e, ecap, ef in zip(experts, ecaps, eflags):
            lo, hi = off[e], off[e + 1]
            if ef >= 0 and hi - lo > ecap:
                ovf[ef] = 1
            for j in range(lo, hi):
                if c >= cap:
                    break
                if unpack:
                    x[j] = b2[c]
                else:
                    b2[c] = x[int(src_rows[j])]
                c += 1
        if sum(off[e + 1] - off[e] for e in experts) > cap and flag >= 0:
            ovf[flag] = 1


XBATCH_MAX_REQ, XBATCH_MAX_GROUPS = 16, 64  # kXbatchMaxReq / kXbatchMaxGroups (kernels.h)


def moe_xbatch_index(offs, reqs, experts, bases, offsets, a_rows):
    """Row map of a cross-request expert batch (one grouped launch for several requests'
    experts): group g = (request ``reqs[g]``, expert ``experts[g]``) takes rows
    [offs[q][e], offs[q][e+1]) of request q's expert-sorted block, which starts at row
    ``bases[q]`` of the batch's token matrix. Writes ``offsets`` (int32 [G+1], prefix sums of
    the groups' device-side counts) and ``a_rows`` (the token row of each sorted row) — one
    workgroup on the GPU, no host sync."""
    if _gpu(offsets):
        ext().moe_xbatch_index(list(offs), list(reqs), list(experts), list(bases), offsets, a_rows)
        return offsets, a_rows
    a_rows.zero_()
    o = 0
    offsets[0] = 0
    for g, (q, e) in enumerate(zip(reqs, experts)):
        lo, hi = int(offs[q][e]), int(offs[q][e + 1])
        a_rows[o:o + hi - lo] = torch.arange(bases[q] + lo, bases[q] + hi, dtype=a_rows.dtype)
        o += hi - lo
        offsets[g + 1] = o
    return offsets, a_rows

def moe_combine(expert_out, slot_of, weights, slot_range=None, out=None):
    """y[m] = sum_j w[m,j] * expert_out[slot_of[m,j]]; with ``slot_range`` (device int32[2])
    only slots in [r0, r1) contribute (one expert's share, zero elsewhere)."""
    if _gpu(expert_out):
        return ext().moe_combine(expert_out.contiguous(), slot_of, weights.contiguous(), slot_range, out)
    M, k = weights.shape
    sl = slot_of.long().reshape(M, k)
    keep = torch.ones_like(sl, dtype=torch.bool)
    if slot_range is not None:
        keep = (sl >= int(slot_range[0])) & (sl < int(slot_range[1]))
    g = expert_out.float()[sl.clamp(0, expert_out.shape[0] - 1).reshape(-1)].reshape(M, k, -1)
    g = torch.where(keep[..., None], g, torch.zeros_like(g))  # rows outside the range are never read
    y = (g * weights.float()[..., None]).sum(1).to(expert_out.dtype)
    return out.copy_(y) if out is not None else y


def moe_gather_combine(experts, idx, slot_of, offsets, gate, residual=None, out=None, ptrs=None, post_norm=None):
    """``out[m] = residual[m] + sum_j gate[m,j] * experts[e][slot[m,j] - offsets[e]]``, e = idx[m,j],
    over COMPACT per-expert outputs (expert e's routed rows at rows 0..count_e-1 of its
    buffer). ``ptrs``: cached int64 device tensor of the expert buffers' addresses (GPU)."""
    M, k = idx.shape
    if _gpu(out):
        if ptrs is None:
            ptrs = torch.tensor([t.data_ptr() for t in experts], dtype=torch.int64, device=out.device)
        o2 = out.view(M, -1)
        return ext().moe_gather_combine([t.reshape(-1, o2.shape[1]) for t in experts], ptrs, idx, slot_of,
                                        offsets, gate.contiguous(), None if residual is None else
                                        residual.reshape(M, -1), o2,
                                        **(_post_norm_args(post_norm) if post_norm is not None else {}))
    H = out.shape[-1]
    acc = residual.reshape(M, H).float().clone() if residual is not None else torch.zeros(M, H)
    off = offsets.long()
    for j in range(k):
        e = idx[:, j].long()
        row = slot_of.reshape(M, k)[:, j].long() - off[e]
        for ee in range(len(experts)):
            sel = (e == ee).nonzero().flatten()
            if sel.numel():
                acc[sel] += gate.reshape(M, k)[sel, j, None].float() * experts[ee].reshape(-1, H)[row[sel]].float()
    out.view(M, H).copy_(acc.to(out.dtype))
    if post_norm is not None:
        _post_norm_ref(out, post_norm)
    return out


def moe_expert(h, router_logits, w_gate_up, w_down, expert, n_experts, top_k, out=None):
    """One expert's contribution for every token (zero where it is not routed): routing
    is recomputed from the router logits, only the expert's routed rows are gathered and
    run through gate_up GEMM -> SwiGLU -> down GEMM (grouped GEMM over a device-side row
    range: no host synchronisation)."""
    idx, gate = moe_router(router_logits, top_k)
    src, slot, off = moe_align(idx, n_experts)
    xp = moe_permute(h, src)
    rng = off[expert:expert + 2].contiguous()
    gu = grouped_gemm(xp, rng, w_gate_up.unsqueeze(0))
    a = swiglu(gu)
    y = grouped_gemm(a, rng, w_down.unsqueeze(0))
    return moe_combine(y, slot, gate, rng, out)


def gemm_grouped(x, weights, offsets, act=None, out=None, outs=None, w_ptrs=None, out_ptrs=None, rows_hint=None,
                 a_rows=None, shared_weights=False):
    """Every expert of an MoE layer in ONE GEMM launch (GPU: LDS-DMA kernel, grid = experts x
    column tiles). Expert e multiplies the expert-sorted rows [offsets[e], offsets[e+1]) of
    ``x`` by ``weights[e]`` ([N][K]; SwiGLU: gate/up-interleaved, N/2 outputs) and writes them
    at the same rows of ``out``, or compactly to rows 0.. of ``outs[e]`` (at most its row
    count). ``a_rows`` (int32 [R]): ``x`` is the TOKEN matrix and sorted row r is token
    ``a_rows[r]`` (the permute happens in the kernel's loads). ``w_ptrs`` / ``out_ptrs``:
    cached int64 device tensors of the tensors' addresses (built here when omitted — pass
    cached ones inside a hipGraph). ``shared_weights``: groups repeat weights (a cross-request
    expert batch) — the launch runs each weight panel's groups together on one XCD and keeps
    the weights cached, so a panel comes from HBM once."""
    a = ACT[act] if not isinstance(act, int) else act
    E = len(weights)
    N, K = weights[0].shape
    R = x.shape[0] if a_rows is None else a_rows.numel()
    if _gpu(x):
        if w_ptrs is None:
            w_ptrs = torch.tensor([w.data_ptr() for w in weights], dtype=torch.int64, device=x.device)
        if outs is not None and out_ptrs is None:
            out_ptrs = torch.tensor([o.data_ptr() for o in outs], dtype=torch.int64, device=x.device)
        hint = rows_hint or max(1, R // E)
        # grouped variants ("g"): tuned as GROUPS experts of `hint` rows in one launch; until
        # tuned, the per-expert row-range choice ("r") stands in
        cfg, _ = tuning.lookup_fused(hint, N, K, ("s" if a == SWIGLU else "") + "g")
        if cfg < 0:
            cfg, _ = tuning.lookup_fused(hint, N, K, tuning.tag(a, True))
        if cfg >= tuning.REGSTAGE:
            cfg = -1
        ext().gemm_grouped(x, list(weights), w_ptrs, offsets, a, out, list(outs) if outs is not None else [],
                           out_ptrs, cfg, a_rows, shared_weights)
        return out if outs is None else outs
    if a_rows is not None:
        x = x[a_rows.long()]
    off = [int(v) for v in offsets.tolist()]
    for e in range(E):
        r0, r1 = off[e], off[e + 1]
        if outs is not None:
            n = min(r1 - r0, outs[e].shape[0])
            if n > 0:
                outs[e][:n] = ref_linear(x[r0:r0 + n], weights[e], act=act)
        elif r1 > r0:
            out[r0:r1] = ref_linear(x[r0:r1], weights[e], act=act)
    return out if outs is None else outs


def grouped_gemm(X, offsets, W, act=None):
    """Per-expert ``act(X_e @ W_e^T)`` over expert-sorted rows; W is [E][N][K]."""
    a = ACT[act] if not isinstance(act, int) else act
    if _gpu(X):
        return ext().grouped_gemm(X.contiguous(), offsets, W.contiguous(), a)
    out = torch.zeros(X.shape[0], W.shape[1], dtype=X.dtype)
    off = offsets.tolist()
    for e in range(W.shape[0]):
        if off[e + 1] > off[e]:
            out[off[e]:off[e + 1]] = ref_linear(X[off[e]:off[e + 1]], W[e], act=a)
    return out
