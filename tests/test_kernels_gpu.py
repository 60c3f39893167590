"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Operands are random (never zero-filled or symmetric); GEMM checks include an
asymmetric-B identity test that catches a transposed C write
(cdna_hip_programming.md §3 "Always A=I-check with ASYMMETRIC B").
"""
import math

import pytest
import torch

from distributed_llm_scheduler_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(*shape, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (scale * torch.randn(*shape, generator=g)).to(dtype).to(DEV)


def _close(a, b, tol):
    err = (a.float() - b.float()).abs().max().item()
    ref = b.float().abs().max().item() + 1e-6
    assert err <= tol * ref, f"max abs err {err:.4g} vs ref max {ref:.4g} (rel tol {tol})"


def test_native_library_loaded():
    m = ops.ext()
    assert hasattr(m, "gemm") and hasattr(m, "attention")


def test_gemm_identity_asymmetric():
    n = 64
    eye = torch.eye(n, dtype=torch.bfloat16, device=DEV)
    b = (torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) % 97 - 48).to(torch.bfloat16)
    # y = I @ W^T = W^T  (W stored [N][K])
    y = ops.linear(eye, b)
    assert torch.equal(y, b.t().contiguous())


@pytest.mark.parametrize("M,N,K", [(512, 2304, 768), (512, 768, 3072), (512, 3072, 768), (77, 130, 200),
                                   (512, 50257, 768), (1, 64, 64), (1024, 1024, 1024)])
@pytest.mark.parametrize("config,splitk", [(-1, 0), (100, 1), (103, 1), (0, 1), (1, 1), (2, 1), (3, 1), (4, 1),
                                           (3, 2), (3, 4), (2, 3), (8, 1), (9, 1), (10, 1), (11, 1), (8, 2),
                                           (12, 1), (13, 1), (14, 1), (15, 1), (12, 2), (14, 4),
                                           (64, 1), (67, 1), (67, 4), (72, 1), (78, 1),  # 64+: persistent
                                           (16, 1), (17, 1), (18, 1), (19, 1), (16, 2), (17, 3), (80, 1),
                                           (20, 1), (21, 1), (21, 3), (22, 1), (23, 1), (24, 1),
                                           (25, 1), (26, 1), (27, 1), (22, 4), (24, 2), (27, 3), (28, 1), (28, 2),
                                           (29, 1), (30, 1), (31, 1), (31, 2), (32, 1), (33, 1), (33, 2),
                                           (34, 1), (35, 1), (34, 2), (34, 3), (98, 1),
                                           (36, 1), (37, 1), (36, 2), (38, 1), (38, 2), (39, 1), (40, 1), (40, 3),
                                           (41, 1), (41, 2), (12, 3), (31, 1), (42, 1), (43, 1), (43, 4), (44, 1), (44, 2), (45, 1),
                                           (46, 1), (46, 2), (47, 1), (47, 3)])
def test_gemm_shapes(M, N, K, config, splitk):
    if K % 64 == 0 and config >= 0 and config < 100 and K % ops.ext().gemm_glds_kstep(config):
        pytest.skip("K-group config needs K % 128 == 0")
    x = _rand(M, K, seed=1)
    w = _rand(N, K, scale=0.05, seed=2)
    ref = ops.ref_linear(x.cpu(), w.cpu()).float()
    y = ops.ext().gemm(x, w, None, None, 0, 1.0, None, config, splitk)
    torch.cuda.synchronize()
    _close(y.cpu(), ref, 2e-2)


@pytest.mark.parametrize("splitk", [1, 2, 4])
def test_gemm_splitk_epilogue(splitk):
    M, N, K = 512, 768, 3072
    x, w = _rand(M, K, seed=30), _rand(N, K, scale=0.02, seed=31)
    bias, res = _rand(N, scale=0.5, seed=32), _rand(M, N, seed=33)
    y = ops.ext().gemm(x, w, bias, res, 1, 1.0, None, 3, splitk)
    ref = ops.ref_linear(x.cpu(), w.cpu(), bias.cpu(), "gelu", res.cpu())
    _close(y.cpu(), ref, 2e-2)


@pytest.mark.parametrize("act", [None, "gelu", "silu"])
def test_gemm_epilogue(act):
    M, N, K = 256, 384, 512
    x, w = _rand(M, K, seed=3), _rand(N, K, scale=0.05, seed=4)
    bias, res = _rand(N, scale=0.5, seed=5), _rand(M, N, seed=6)
    y = ops.linear(x, w, bias=bias, act=act, residual=res)
    ref = ops.ref_linear(x.cpu(), w.cpu(), bias.cpu(), act, res.cpu())
    _close(y.cpu(), ref, 2e-2)


@pytest.mark.parametrize("B,S,nh,nkv,D,causal", [(1, 512, 12, 12, 64, True), (2, 200, 4, 4, 64, True),
                                                  (1, 256, 8, 2, 128, True), (1, 130, 4, 4, 64, False),
                                                  (1, 64, 32, 8, 128, True)])
@pytest.mark.parametrize("variant", list(range(15)))
def test_attention(B, S, nh, nkv, D, causal, variant):
    qkv = _rand(B * S, (nh + 2 * nkv) * D, seed=7)
    q, k, v = qkv[:, :nh * D], qkv[:, nh * D:(nh + nkv) * D], qkv[:, (nh + nkv) * D:]
    o = ops.ext().attention(q, k, v, B, S, nh, nkv, D, causal, 1.0 / math.sqrt(D), None, variant)
    ref = ops.ref_attention(q.cpu(), k.cpu(), v.cpu(), B, S, nh, nkv, D, causal=causal)
    _close(o.cpu(), ref, 2e-2)


@pytest.mark.parametrize("B,S,Sq,q_off,nh,nkv,D", [(1, 512, 128, 384, 12, 12, 64), (2, 256, 64, 64, 4, 4, 64),
                                                    (1, 512, 256, 256, 32, 8, 128), (1, 200, 50, 150, 4, 2, 128),
                                                    (1, 384, 128, 0, 12, 12, 64)])
def test_attention_query_chunk(B, S, Sq, q_off, nh, nkv, D):
    # a sequence chunk's queries (positions q_off..) against every key before them:
    # the attention node of the sequence-parallel DAG transform
    kv = _rand(B * S, 2 * nkv * D, seed=71)
    q = _rand(B * Sq, nh * D, seed=72)
    k, v = kv[:, :nkv * D], kv[:, nkv * D:]
    o = ops.attention(q, k, v, B, S, nh, nkv, D, True, Sq=Sq, q_off=q_off)
    ref = ops.ref_attention(q.cpu(), k.cpu(), v.cpu(), B, S, nh, nkv, D, True, Sq=Sq, q_off=q_off)
    _close(o.cpu(), ref, 2e-2)


def test_attention_spike_forces_rescale():
    # a large score late in the sequence forces the online-softmax rescale branch
    B, S, nh, D = 1, 256, 2, 64
    qkv = _rand(B * S, 3 * nh * D, scale=0.5, seed=8)
    qkv[:, nh * D:2 * nh * D][200] *= 40.0
    q, k, v = qkv[:, :nh * D], qkv[:, nh * D:2 * nh * D], qkv[:, 2 * nh * D:]
    o = ops.attention(q, k, v, B, S, nh, nh, D)
    ref = ops.ref_attention(q.cpu(), k.cpu(), v.cpu(), B, S, nh, nh, D)
    _close(o.cpu(), ref, 3e-2)


@pytest.mark.parametrize("H", [64, 768, 1024, 2048, 4096, 5120, 8192])
def test_layernorm_and_residual(H):
    x, r = _rand(300, H, seed=9), _rand(300, H, seed=10)
    w, b = (1 + 0.1 * _rand(H, seed=11).float()).to(torch.bfloat16), _rand(H, scale=0.1, seed=12)
    y = ops.layernorm(x, w, b)
    _close(y.cpu(), ops.ref_layernorm(x.cpu(), w.cpu(), b.cpu()), 2e-2)
    y2, s = ops.layernorm(x, w, b, residual=r)
    s_ref = (x.cpu().float() + r.cpu().float()).to(torch.bfloat16)
    assert torch.equal(s.cpu(), s_ref)
    _close(y2.cpu(), ops.ref_layernorm(s_ref, w.cpu(), b.cpu()), 2e-2)


@pytest.mark.parametrize("M,H", [(100, 4096), (301, 4096), (7, 768), (513, 8192), (3, 2048)])
def test_rmsnorm(M, H):
    x, w = _rand(M, H, seed=13), (1 + 0.1 * _rand(H, seed=14).float()).to(torch.bfloat16)
    _close(ops.rmsnorm(x, w).cpu(), ops.ref_rmsnorm(x.cpu(), w.cpu()), 2e-2)
    r = _rand(M, H, seed=15)
    y, s = ops.rmsnorm(x, w, residual=r)
    s_ref = (x.cpu().float() + r.cpu().float()).to(torch.bfloat16)
    assert torch.equal(s.cpu(), s_ref)
    _close(y.cpu(), ops.ref_rmsnorm(s_ref, w.cpu()), 2e-2)


def test_elementwise():
    x, y = _rand(1000, 64, seed=15), _rand(1000, 64, seed=16)
    _close(ops.gelu(x).cpu(), torch.nn.functional.gelu(x.cpu().float(), approximate="tanh"), 1e-2)
    _close(ops.add(x, y).cpu(), x.cpu().float() + y.cpu().float(), 1e-2)
    gu = _rand(50, 2 * 96, seed=17)
    ref = torch.nn.functional.silu(gu.cpu().float()[:, :96]) * gu.cpu().float()[:, 96:]
    _close(ops.swiglu(gu).cpu(), ref, 1e-2)


def test_embedding():
    V, H, S = 1000, 256, 64
    wte, wpe = _rand(V, H, seed=18), _rand(S, H, seed=19)
    tok = torch.randint(0, V, (2 * S,), device=DEV, dtype=torch.int32)
    y = ops.embedding(tok, wte, wpe, S)
    ref = ops.embedding(tok.cpu(), wte.cpu(), wpe.cpu(), S)
    _close(y.cpu(), ref, 1e-2)


@pytest.mark.parametrize("D", [64, 128])
def test_rope(D):
    S, nh, nkv = 64, 4, 2
    qkv = _rand(2 * S, (nh + 2 * nkv) * D, seed=20)
    cos, sin = ops.rope_tables(S, D, 10000.0, DEV)
    ref = ops.ref_rope_(qkv.cpu().clone(), S, nh, nkv, D, nh * D, cos.cpu(), sin.cpu())
    ops.rope_(qkv, S, nh, nkv, D, nh * D, cos, sin)
    _close(qkv.cpu(), ref, 1e-2)


def test_moe_pipeline():
    M, E, k, H, F = 300, 8, 2, 128, 96
    # tie-free logits (bf16 random values collide; top-k order among ties is unspecified)
    g = torch.Generator().manual_seed(21)
    logits = torch.stack([torch.randperm(E, generator=g) for _ in range(M)]).float().mul(0.25)
    logits = logits.to(torch.bfloat16).to(DEV)
    idx, w = ops.moe_router(logits, k)
    ridx, rw = ops.moe_router(logits.cpu(), k)
    assert torch.equal(idx.cpu().sort(-1).values, ridx.sort(-1).values)
    src, slot, off = ops.moe_align(idx, E)
    rsrc, rslot, roff = ops.moe_align(idx.cpu(), E)
    assert torch.equal(off.cpu(), roff) and torch.equal(src.cpu(), rsrc) and torch.equal(slot.cpu(), rslot)
    x = _rand(M, H, seed=22)
    xp = ops.moe_permute(x, src)
    assert torch.equal(xp.cpu(), x.cpu()[rsrc.long()])
    W = _rand(E, F, H, scale=0.05, seed=23)
    y = ops.grouped_gemm(xp, off, W, act="silu")
    yr = ops.grouped_gemm(xp.cpu(), roff, W.cpu(), act="silu")
    _close(y.cpu(), yr, 2e-2)
    eo = _rand(M * k, H, seed=24)
    _close(ops.moe_combine(eo, slot, w).cpu(), ops.moe_combine(eo.cpu(), slot.cpu(), w.cpu()), 1e-2)


@pytest.mark.parametrize("mode", ["layernorm", "rmsnorm"])
@pytest.mark.parametrize("M,N,K,cfg", [(512, 2304, 768, -1), (300, 1024, 4096, 0), (512, 3072, 768, 2),
                                       (512, 1024, 1024, 8), (256, 512, 768, 14),
                                       (512, 2304, 768, 67), (512, 3072, 768, 64), (512, 768, 768, 16),
                                       (512, 3072, 768, 22), (512, 2304, 768, 23), (512, 768, 768, 24)])
def test_gemm_with_folded_norm(mode, M, N, K, cfg):
    x = _rand(M, K, scale=2.0, seed=40) + 0.5  # non-zero mean rows exercise the mean correction
    w = _rand(N, K, scale=0.03, seed=41)
    nw = (1 + 0.2 * _rand(K, seed=42).float()).to(torch.bfloat16)
    nb = _rand(K, scale=0.1, seed=43) if mode == "layernorm" else None
    bias = _rand(N, scale=0.1, seed=44)
    res = _rand(M, N, seed=45)
    if mode == "layernorm":
        xn = ops.ref_layernorm(x.cpu(), nw.cpu(), nb.cpu())
    else:
        xn = ops.ref_rmsnorm(x.cpu(), nw.cpu())
    ref = ops.ref_linear(xn, w.cpu(), bias.cpu(), "gelu", res.cpu())
    wd, cs, bd = ops.derive_norm_gemm(w, nw, nb, bias)
    y = ops.linear_norm(x, wd, cs, bd, mode, act="gelu", residual=res)
    _close(y.cpu(), ref, 3e-2)
    y2 = ops.ext().gemm(x, wd, bd, res, 1, 1.0, None, cfg, 1, cs, 1 if mode == "layernorm" else 2, 1e-5)
    _close(y2.cpu(), ref, 3e-2)


def _ref_swiglu(x, w13, bias=None):
    F = w13.shape[0] // 2
    y = x.float() @ w13.float().t()
    if bias is not None:
        y = y + bias.float()
    return torch.nn.functional.silu(y[:, :F]) * y[:, F:]


@pytest.mark.parametrize("config,splitk", [(-1, 0), (0, 1), (3, 1), (3, 4), (8, 1), (7, 2), (2, 1), (12, 1),
                                           (14, 2), (15, 1), (17, 1), (16, 2), (21, 1), (22, 1), (25, 2),
                                           (37, 1), (37, 2), (40, 1), (36, 1)])
@pytest.mark.parametrize("M,F,K", [(512, 1024, 768), (200, 512, 1024), (64, 96, 128)])
def test_gemm_swiglu_epilogue(M, F, K, config, splitk):
    if config >= 16 and K % (ops.ext().gemm_glds_kstep(config) * splitk):
        pytest.skip("K-group config needs K % 128 == 0 per split")
    if K % (64 * max(splitk, 1)):
        pytest.skip("split does not divide K")
    x = _rand(M, K, seed=50)
    w13 = _rand(2 * F, K, scale=0.05, seed=51)
    b13 = _rand(2 * F, scale=0.2, seed=52)
    ref = _ref_swiglu(x.cpu(), w13.cpu(), b13.cpu())
    y = ops.ext().gemm(x, ops.interleave_gate_up(w13), ops.interleave_gate_up(b13), None, ops.SWIGLU, 1.0, None,
                       config, splitk)
    torch.cuda.synchronize()
    assert y.shape == (M, F)
    _close(y.cpu(), ref, 2e-2)
    # the CPU reference path of the same op agrees too
    yc = ops.linear(x.cpu(), ops.interleave_gate_up(w13.cpu()), ops.interleave_gate_up(b13.cpu()), act="swiglu")
    _close(yc, ref, 2e-2)


@pytest.mark.parametrize("act", [None, "swiglu"])
@pytest.mark.parametrize("config,splitk", [(-1, 0), (3, 1), (7, 1), (3, 4), (0, 2), (12, 1), (15, 2),
                                           (17, 1), (16, 2), (20, 1), (22, 1), (25, 1)])
@pytest.mark.parametrize("r0,r1", [(100, 229), (0, 512), (300, 300), (448, 512)])
def test_gemm_row_range(act, config, splitk, r0, r1):
    M, N, K = 512, 1024, 1024
    x = _rand(M, K, seed=60)
    w = _rand(N, K, scale=0.05, seed=61)
    wk = ops.interleave_gate_up(w) if act else w
    no = N // 2 if act else N
    out = torch.full((M, no), 7.0, dtype=torch.bfloat16, device=DEV)
    rows = torch.tensor([r0, r1], dtype=torch.int32, device=DEV)
    ops.ext().gemm(x, wk, None, None, ops.ACT[act], 1.0, out, config, splitk, None, 0, 1e-5, rows)
    torch.cuda.synchronize()
    o = out.cpu().float()
    assert (o[:r0] == 7.0).all() and (o[r1:] == 7.0).all(), "rows outside the range were written"
    if r1 > r0:
        ref = _ref_swiglu(x[r0:r1].cpu(), w.cpu()) if act else ops.ref_linear(x[r0:r1].cpu(), w.cpu()).float()
        _close(o[r0:r1], ref, 2e-2)


@pytest.mark.parametrize("mode", ["layernorm", "rmsnorm"])
def test_folded_norm_with_swiglu(mode):
    M, F, K = 256, 512, 512
    x = _rand(M, K, scale=2.0, seed=70) + 0.3
    w13 = _rand(2 * F, K, scale=0.04, seed=71)
    nw = (1 + 0.2 * _rand(K, seed=72).float()).to(torch.bfloat16)
    nb = _rand(K, scale=0.1, seed=73) if mode == "layernorm" else None
    xn = ops.ref_layernorm(x.cpu(), nw.cpu(), nb.cpu()) if mode == "layernorm" else ops.ref_rmsnorm(x.cpu(), nw.cpu())
    ref = _ref_swiglu(xn, w13.cpu())
    wd, cs, bd = ops.derive_norm_gemm(w13, nw, nb, None)
    wi, csi = ops.interleave_gate_up(wd), ops.interleave_gate_up(cs)
    bi = ops.interleave_gate_up(bd) if nb is not None else None
    y = ops.linear_norm(x, wi, csi, bi, mode, act="swiglu")
    _close(y.cpu(), ref, 3e-2)


@pytest.mark.parametrize("config,splitk", [(-1, 0), (7, 1), (15, 4), (3, 2)])
def test_gemm_row_range_compact(config, splitk):
    M, N, K, cap = 512, 512, 1024, 200
    x = _rand(M, K, seed=80)
    w = _rand(N, K, scale=0.05, seed=81)
    out = torch.full((cap, N), 7.0, dtype=torch.bfloat16, device=DEV)
    rows = torch.tensor([130, 290], dtype=torch.int32, device=DEV)  # 160 rows -> out rows 0..159
    ops.ext().gemm(x, w, None, None, 0, 1.0, out, config, splitk, None, 0, 1e-5, rows, True)
    torch.cuda.synchronize()
    o = out.cpu().float()
    _close(o[:160], ops.ref_linear(x[130:290].cpu(), w.cpu()).float(), 2e-2)
    assert (o[160:] == 7.0).all()
    over = torch.tensor([0, 400], dtype=torch.int32, device=DEV)  # more rows than the output holds: clamped
    ops.ext().gemm(x, w, None, None, 0, 1.0, out, config, splitk, None, 0, 1e-5, over, True)
    torch.cuda.synchronize()
    _close(out.cpu().float(), ops.ref_linear(x[:cap].cpu(), w.cpu()).float(), 2e-2)


@pytest.mark.parametrize("config", [-1, 3, 15, 17, 25, 1, 28, 29, 30, 31, 32, 33, 41, 37, 44, 46, 47])
def test_gemm_grouped_experts(config):
    """All experts of a layer in one launch: SwiGLU gate/up into shared rows, then the down
    GEMM into per-expert compact outputs — against per-expert fp32 references."""
    E, H, F, R = 4, 256, 384, 300
    counts = [70, 0, 130, 100]
    off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=DEV)
    x = _rand(R, H, seed=90)
    w13 = [ops.interleave_gate_up(_rand(2 * F, H, scale=0.05, seed=91 + e)) for e in range(E)]
    w2 = [_rand(H, F, scale=0.05, seed=95 + e) for e in range(E)]
    h = torch.full((R, F), 5.0, dtype=torch.bfloat16, device=DEV)
    cap = 120
    outs = [torch.full((cap, H), 7.0, dtype=torch.bfloat16, device=DEV) for _ in range(E)]
    ext = ops.ext()
    wp13 = torch.tensor([w.data_ptr() for w in w13], dtype=torch.int64, device=DEV)
    wp2 = torch.tensor([w.data_ptr() for w in w2], dtype=torch.int64, device=DEV)
    op = torch.tensor([o.data_ptr() for o in outs], dtype=torch.int64, device=DEV)
    ext.gemm_grouped(x, w13, wp13, off, 4, h, [], None, config)
    ext.gemm_grouped(h, w2, wp2, off, 0, None, outs, op, config)
    torch.cuda.synchronize()
    o = off.tolist()
    for e in range(E):
        r0, r1 = o[e], o[e + 1]
        if r1 > r0:
            href = ops.ref_linear(x[r0:r1].cpu(), w13[e].cpu(), act="swiglu")
            _close(h[r0:r1].cpu(), href.float(), 2e-2)
            n = min(r1 - r0, cap)
            _close(outs[e][:n].cpu(), ops.ref_linear(h[r0:r0 + n].cpu(), w2[e].cpu()).float(), 2e-2)
        assert (outs[e][min(r1 - r0, cap):].cpu().float() == 7.0).all(), "rows past the expert's count were written"


@pytest.mark.parametrize("tall", ["0", "1"])
@pytest.mark.parametrize("xcd", ["0", "1"])
@pytest.mark.parametrize("pairs", ["0", "1", "2", "3"])
@pytest.mark.parametrize("config", [-1, 17, 31, 33, 41, 44, 46])
def test_gemm_grouped_heavy_expert(config, pairs, xcd, tall, monkeypatch):
    """Experts with several row tiles (450 rows: three 160-row tiles, three 192-row tiles, eight
    64-row tiles) next to tiny and empty ones: the row-split pairs of a grouped launch (even row
    tiles in one block, odd in its same-XCD partner) cover every row exactly once — against
    per-expert fp32 references, untouched rows past the last expert. DLS_EXPERT_PAIRS: 0 one
    block walks all of (expert, column panel)'s row tiles, 1 same-XCD partner blocks, 2 partners
    in the grid's second half (the default), 3 in its first half; DLS_EXPERT_XCD=1 the XCD-affine
    block order (6 groups: not a multiple of the 8 XCDs); DLS_EXPERT_TALL=1 one taller tile for an
    expert within it (config 33's 192 rows -> 256 and config 44's 160 -> 224: the 161- and 200-row experts)."""
    monkeypatch.setenv("DLS_EXPERT_PAIRS", pairs)
    monkeypatch.setenv("DLS_EXPERT_XCD", xcd)
    monkeypatch.setenv("DLS_EXPERT_TALL", tall)
    H, F = 256, 384
    counts = [20, 450, 0, 200, 7, 161]
    E, R = len(counts), sum(counts) + 16
    off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=DEV)
    x = _rand(R, H, seed=190)
    w13 = [ops.interleave_gate_up(_rand(2 * F, H, scale=0.05, seed=191 + e)) for e in range(E)]
    w2 = [_rand(H, F, scale=0.05, seed=201 + e) for e in range(E)]
    h = torch.full((R, F), 5.0, dtype=torch.bfloat16, device=DEV)
    y = torch.full((R, H), 7.0, dtype=torch.bfloat16, device=DEV)
    ext = ops.ext()
    wp13 = torch.tensor([w.data_ptr() for w in w13], dtype=torch.int64, device=DEV)
    wp2 = torch.tensor([w.data_ptr() for w in w2], dtype=torch.int64, device=DEV)
    ext.gemm_grouped(x, w13, wp13, off, 4, h, [], None, config)
    ext.gemm_grouped(h, w2, wp2, off, 0, y, [], None, config)
    # the gate/up launch gathering its rows from a token matrix (the Mixtral step's form): sorted
    # row r reads token a_rows[r]
    n = sum(counts)
    g = torch.Generator().manual_seed(5)
    a_rows = torch.randint(0, 300, (n,), generator=g).to(torch.int32).to(DEV)
    tok = _rand(300, H, seed=189)
    hg = torch.full((n, F), 3.0, dtype=torch.bfloat16, device=DEV)  # (out rows = a_rows' count)
    ext.gemm_grouped(tok, w13, wp13, off, 4, hg, [], None, config, a_rows)
    torch.cuda.synchronize()
    o = off.tolist()
    xs = tok.cpu()[a_rows.cpu().long()]
    for e in range(E):
        r0, r1 = o[e], o[e + 1]
        if r1 > r0:
            href = ops.ref_linear(x[r0:r1].cpu(), w13[e].cpu(), act="swiglu")
            _close(h[r0:r1].cpu(), href.float(), 2e-2)
            _close(y[r0:r1].cpu(), ops.ref_linear(h[r0:r1].cpu(), w2[e].cpu()).float(), 2e-2)
            _close(hg[r0:r1].cpu(), ops.ref_linear(xs[r0:r1], w13[e].cpu(), act="swiglu").float(), 2e-2)
    assert (h[o[-1]:].cpu().float() == 5.0).all() and (y[o[-1]:].cpu().float() == 7.0).all()


@pytest.mark.parametrize("M,E,k", [(300, 8, 2), (512, 8, 2), (1500, 8, 2), (200, 64, 8), (777, 16, 1)])
def test_moe_route_fused_equals_router_align(M, E, k):
    """The one-workgroup route kernel returns exactly what moe_router + moe_align return."""
    g = torch.Generator().manual_seed(M + E)
    logits = torch.stack([torch.randperm(E, generator=g) for _ in range(M)]).float().mul(0.25)
    logits = (logits + 0.01 * torch.randn(M, E, generator=g)).to(torch.bfloat16).to(DEV)
    idx, w = ops.moe_router(logits, k)
    src, slot, off = ops.moe_align(idx, E)
    fi, fw, fs, fsl, fo = ops.ext().moe_route(logits, k)
    torch.cuda.synchronize()
    assert torch.equal(fi, idx) and torch.equal(fw, w)
    assert torch.equal(fo, off) and torch.equal(fs, src) and torch.equal(fsl, slot)


@pytest.mark.parametrize("M,E,k,H", [(512, 8, 2, 4096), (300, 8, 2, 256), (100, 16, 4, 512), (77, 64, 2, 128)])
def test_moe_gate_route_fused(M, E, k, H):
    """Router GEMM + routing in one launch (last workgroup routes): logits match the fp32
    reference, and the routing equals moe_route over those same logits. E = 64 takes the
    GEMM + moe_route fallback."""
    x = _rand(M, H, seed=7)
    wg = _rand(E, H, scale=0.05, seed=8)
    logits = torch.empty(M, E, dtype=torch.bfloat16, device=DEV)
    for _ in range(3):  # repeated launches: the ticket must be reset by every last block
        r = ops.moe_gate_route(x, wg, k, logits)
    torch.cuda.synchronize()
    _close(logits.cpu().float(), ops.ref_linear(x.cpu(), wg.cpu()).float(), 2e-2)
    ref = ops.moe_route(logits, k, E)
    torch.cuda.synchronize()
    for a, b in zip(r, ref):
        assert torch.equal(a, b)


def test_moe_gate_route_many_blocks():
    """The one-launch router hands the logits of 1024 workgroups to the last arriver without a
    fence (sc1 stores / ticket / sc1 loads): at the largest M the fused kernel takes, with new
    logits every launch (the last block's L1 still holds the previous launch's lines) and a GEMM
    on another stream loading the chip unevenly, the routing equals moe_route over the logits
    written."""
    M, E, k, H = 2048, 8, 2, 1024
    wg = _rand(E, H, scale=0.05, seed=8)
    logits = torch.empty(M, E, dtype=torch.bfloat16, device=DEV)
    side = torch.cuda.Stream()
    a, b = _rand(4096, 4096, seed=1), _rand(4096, 4096, seed=2)
    for it in range(8):
        x = _rand(M, H, seed=100 + it)
        with torch.cuda.stream(side):
            torch.matmul(a, b)
        r = ops.moe_gate_route(x, wg, k, logits)
        torch.cuda.synchronize()
        assert r is not None
        ref = ops.moe_route(logits, k, E)
        torch.cuda.synchronize()
        for u, v in zip(r, ref):
            assert torch.equal(u, v), f"launch {it}: routing differs from the published logits"
        _close(logits.cpu().float(), ops.ref_linear(x.cpu(), wg.cpu()).float(), 2e-2)


@pytest.mark.parametrize("config", [-1, 3, 17, 30, 31, 33, 41, 44, 46, 47])
def test_gemm_grouped_gathered_rows(config):
    """Gate/up grouped GEMM reading its expert-sorted rows straight from the token matrix
    (a_rows = src rows of the routing) equals the permute-then-GEMM path."""
    M, E, k, H, F = 300, 8, 2, 256, 384
    g = torch.Generator().manual_seed(5)
    logits = torch.stack([torch.randperm(E, generator=g) for _ in range(M)]).float().to(torch.bfloat16).to(DEV)
    idx, gate, src, slot, off = ops.moe_route(logits, k, E)
    x = _rand(M, H, seed=31)
    w13 = [ops.interleave_gate_up(_rand(2 * F, H, scale=0.05, seed=40 + e)) for e in range(E)]
    R = src.numel()
    h_ref = torch.zeros(R, F, dtype=torch.bfloat16, device=DEV)
    h = torch.full((R, F), 3.0, dtype=torch.bfloat16, device=DEV)
    ops.gemm_grouped(ops.moe_permute(x, src), w13, off, act="swiglu", out=h_ref)
    ops.gemm_grouped(x, w13, off, act="swiglu", out=h, a_rows=src)
    ext = ops.ext()
    wp = torch.tensor([w.data_ptr() for w in w13], dtype=torch.int64, device=DEV)
    h2 = torch.full((R, F), 3.0, dtype=torch.bfloat16, device=DEV)
    ext.gemm_grouped(x, w13, wp, off, 4, h2, [], None, config, src)
    torch.cuda.synchronize()
    assert torch.equal(h, h_ref)
    xs = x.cpu()[src.cpu().long()]
    o = off.tolist()
    for e in range(E):
        r0, r1 = o[e], o[e + 1]
        if r1 > r0:
            _close(h2[r0:r1].cpu(), ops.ref_linear(xs[r0:r1], w13[e].cpu(), act="swiglu").float(), 2e-2)


def test_moe_gather_combine():
    M, E, k, H = 300, 8, 2, 256
    g = torch.Generator().manual_seed(90)
    logits = torch.randn(M, E, generator=g).to(torch.bfloat16)
    idx, gate = ops.moe_router(logits, k)
    src, slot, off = ops.moe_align(idx, E)
    counts = (off[1:] - off[:-1]).tolist()
    experts = [(torch.randn(M, H, generator=g) * (1 + e)).to(torch.bfloat16) for e in range(E)]
    res = torch.randn(M, H, generator=g).to(torch.bfloat16)
    ref = ops.moe_gather_combine(experts, idx, slot, off, gate, residual=res, out=torch.empty(M, H, dtype=torch.bfloat16))
    # explicit fp32 recomputation
    exp = res.float().clone()
    for m in range(M):
        for j in range(k):
            e = int(idx[m, j])
            exp[m] += float(gate[m, j]) * experts[e][int(slot[m * k + j]) - int(off[e])].float()
    _close(ref.float(), exp, 1e-2)
    assert all(c <= M for c in counts)
    out = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    y = ops.moe_gather_combine([t.to(DEV) for t in experts], idx.to(DEV), slot.to(DEV), off.to(DEV), gate.to(DEV),
                               residual=res.to(DEV), out=out)
    torch.cuda.synchronize()
    _close(y.cpu().float(), exp, 1e-2)


def test_moe_gather_combine_no_nan_from_unused_rows():
    """Top-3 (padded expert slots) and no residual: the padding slots and every row past an
    expert's routed count hold Inf, the output buffer holds NaN before the launch — none of it
    may leak into the combined rows (unused loads are discarded by select, not weighted by 0)."""
    M, E, k, H = 257, 8, 3, 512
    g = torch.Generator().manual_seed(91)
    logits = torch.randn(M, E, generator=g).to(torch.bfloat16)
    idx, gate = ops.moe_router(logits, k)
    src, slot, off = ops.moe_align(idx, E)
    counts = (off[1:] - off[:-1]).tolist()
    experts = []
    for e in range(E):
        t = torch.randn(M, H, generator=g).to(torch.bfloat16)
        t[counts[e]:] = float("inf")
        experts.append(t)
    exp = torch.zeros(M, H)
    for m in range(M):
        for j in range(k):
            e = int(idx[m, j])
            exp[m] += float(gate[m, j]) * experts[e][int(slot[m * k + j]) - int(off[e])].float()
    out = torch.full((M, H), float("nan"), dtype=torch.bfloat16, device=DEV)
    y = ops.moe_gather_combine([t.to(DEV) for t in experts], idx.to(DEV), slot.to(DEV), off.to(DEV), gate.to(DEV),
                               residual=None, out=out)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(y.float()).all())
    _close(y.cpu().float(), exp, 1e-2)


@pytest.mark.parametrize("config,splitk", [(-1, 0), (3, 1), (0, 2), (3, 4), (8, 1)])
def test_gemm_rope_epilogue(config, splitk):
    B, S, nh, nkv, D, H = 2, 128, 4, 2, 128, 512
    M, width = B * S, (nh + 2 * nkv) * D
    x = _rand(M, H, seed=95)
    w = _rand(width, H, scale=0.05, seed=96)
    b = _rand(width, scale=0.1, seed=97)
    cos, sin = ops.rope_tables(S, D, 10000.0, DEV)
    perm = ops.rope_pair_perm(nh, nkv, D, width).to(DEV)
    rope = (cos, sin, S, D, (nh + nkv) * D)
    y = ops.ext().gemm(x, w[perm].contiguous(), b[perm].contiguous(), None, 0, 1.0, None, config, splitk, None, 0,
                       1e-5, None, False, cos, sin, S, D, (nh + nkv) * D)
    torch.cuda.synchronize()
    ref = ops.ref_linear(x.cpu(), w[perm].cpu(), b[perm].cpu(), rope=(cos.cpu(), sin.cpu(), S, D, (nh + nkv) * D))
    _close(y.cpu(), ref.float(), 2e-2)
    # attention over the pair-interleaved q/k equals attention with standard rotate-half RoPE
    std = ops.ref_linear(x.cpu(), w.cpu(), b.cpu())
    ops.ref_rope_(std, S, nh, nkv, D, nh * D, cos.cpu(), sin.cpu())
    split = lambda t: (t[:, :nh * D], t[:, nh * D:(nh + nkv) * D], t[:, (nh + nkv) * D:])  # noqa: E731
    o_std = ops.ref_attention(*split(std), B, S, nh, nkv, D, causal=True)
    o_new = ops.ref_attention(*split(y.cpu()), B, S, nh, nkv, D, causal=True)
    _close(o_new, o_std.float(), 3e-2)


@pytest.mark.parametrize("N", [768, 4096])
@pytest.mark.parametrize("config,splitk", [(3, 1), (3, 3), (0, 1), (8, 2), (100, 1), (34, 1), (34, 2)])
def test_gemm_emits_row_stats(config, splitk, N):
    M, K = 300, 768
    x, w = _rand(M, K, seed=100), _rand(N, K, scale=0.05, seed=101)
    b, r = _rand(N, scale=0.1, seed=102), _rand(M, N, seed=103)
    st = torch.zeros(M, 2, dtype=torch.float32, device=DEV)
    y = ops.ext().gemm(x, w, b, r, 0, 1.0, None, config, splitk, None, 0, 1e-5, None, False, None, None, 1, 2, 0,
                       st, None)
    torch.cuda.synchronize()
    yf = y.cpu().float()
    ref = torch.stack([yf.sum(1), (yf * yf).sum(1)], 1)
    assert torch.allclose(st.cpu(), ref, rtol=1e-4, atol=1e-2), (st.cpu() - ref).abs().max()


@pytest.mark.parametrize("mode", ["layernorm", "rmsnorm"])
@pytest.mark.parametrize("config,splitk,act", [(3, 1, 0), (3, 4, 1), (0, 2, 0), (8, 1, 0), (12, 2, 0), (3, 1, 4),
                                               (34, 1, 0), (34, 2, 1), (35, 1, 0),
                                               (36, 1, 0), (37, 1, 4), (38, 1, 0), (39, 2, 0), (40, 1, 1),
                                               (42, 1, 0)])
def test_gemm_folded_norm_external_stats(mode, config, splitk, act):
    M, N, K = 256, 1024, 2048
    x = _rand(M, K, scale=2.0, seed=110) + 0.3
    w = _rand(N, K, scale=0.03, seed=111)
    nw = (1 + 0.2 * _rand(K, seed=112).float()).to(torch.bfloat16)
    nb = _rand(K, scale=0.1, seed=113) if mode == "layernorm" else None
    xf = x.cpu().float()
    st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).to(DEV)
    xn = ops.ref_layernorm(x.cpu(), nw.cpu(), nb.cpu()) if mode == "layernorm" else ops.ref_rmsnorm(x.cpu(), nw.cpu())
    wd, cs, bd = ops.derive_norm_gemm(w, nw, nb, None)
    if act == 4:  # SwiGLU epilogue over the folded, interleaved weight
        ref = _ref_swiglu(xn, w.cpu())
        wd, cs = ops.interleave_gate_up(wd), ops.interleave_gate_up(cs)
        bd = ops.interleave_gate_up(bd) if nb is not None else None
    else:
        ref = ops.ref_linear(xn, w.cpu(), act=act).float()
        bd = bd if nb is not None else None
    y = ops.ext().gemm(x, wd, bd, None, act, 1.0, None, config, splitk, cs, 1 if mode == "layernorm" else 2, 1e-5,
                       None, False, None, None, 1, 2, 0, None, st)
    torch.cuda.synchronize()
    _close(y.cpu(), ref, 3e-2)


@pytest.mark.parametrize("nbytes,blocks", [(256, 1), (6144, 64), (1 << 20, 128), ((9 << 20) + 4096, 512)])
def test_host_pull_copies_exact_bytes(nbytes, blocks):
    """Parameter refill by the host-pull kernel: pinned host image -> HBM, bit-exact, and
    nothing past the destination prefix is written."""
    g = torch.Generator().manual_seed(nbytes)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, generator=g).pin_memory()
    dst = torch.full((nbytes + 4096,), 0xA5, dtype=torch.uint8, device=DEV)
    ops.ext().host_pull(dst, src, blocks)
    torch.cuda.synchronize()
    assert torch.equal(dst[:nbytes].cpu(), src)
    assert bool((dst[nbytes:] == 0xA5).all())


@pytest.mark.parametrize("mode", ["rmsnorm", "layernorm"])
@pytest.mark.parametrize("config,splitk", [(0, 4), (14, 4), (0, 2), (3, 1), (100, 1)])
def test_gemm_post_norm(mode, config, splitk):
    """A residual GEMM that also writes the next norm of its output rows: split-K launches do it
    in the row-owning reduce, the others with the norm kernel after the GEMM. The output equals
    the plain GEMM's bit for bit; the normalised rows match the norm kernel on that output."""
    M, N, K = 512, 4096, 1024
    x = _rand(M, K, seed=60)
    w = _rand(N, K, scale=0.03, seed=61)
    res = _rand(M, N, seed=62)
    nw = (1 + 0.2 * _rand(N, seed=63).float()).to(torch.bfloat16)
    nb = _rand(N, scale=0.1, seed=64) if mode == "layernorm" else None
    plain = ops.ext().gemm(x, w, None, res, 0, 1.0, None, config, splitk)
    yn = torch.full((M, N), 9.0, dtype=torch.bfloat16, device=DEV)
    out = ops.ext().gemm(x, w, None, res, 0, 1.0, None, config, splitk, norm_out=yn, norm_w=nw, norm_b=nb,
                         norm_mode=1 if mode == "layernorm" else 2, norm_eps=1e-5)
    ref_n = ops.layernorm(plain, nw, nb) if mode == "layernorm" else ops.rmsnorm(plain, nw)
    torch.cuda.synchronize()
    assert torch.equal(out, plain)
    _close(yn.cpu().float(), ref_n.cpu().float(), 2e-2)


def test_moe_gather_combine_post_norm():
    M, E, k, H = 300, 8, 2, 4096
    g = torch.Generator().manual_seed(91)
    logits = torch.randn(M, E, generator=g).to(torch.bfloat16).to(DEV)
    idx, gate, src, slot, off = ops.moe_route(logits, k, E)
    experts = [(torch.randn(M, H, generator=g) * 0.5).to(torch.bfloat16).to(DEV) for _ in range(E)]
    res = torch.randn(M, H, generator=g).to(torch.bfloat16).to(DEV)
    nw = (1 + 0.2 * _rand(H, seed=92).float()).to(torch.bfloat16)
    out = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    yn = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    ops.moe_gather_combine(experts, idx, slot, off, gate, residual=res, out=out, post_norm=(yn, nw, None, "rmsnorm", 1e-5))
    plain = torch.empty_like(out)
    ops.moe_gather_combine(experts, idx, slot, off, gate, residual=res, out=plain)
    ref_n = ops.rmsnorm(plain, nw)
    torch.cuda.synchronize()
    assert torch.equal(out, plain)
    _close(yn.cpu().float(), ref_n.cpu().float(), 2e-2)


@pytest.mark.parametrize("split", [True, False])
def test_lm_head_column_split(split, monkeypatch):
    """The GPT-2 LM head as the DAG runs it (512 x 50257 x 768, final LayerNorm folded, row
    statistics handed over, logits written into rows padded to 50304): one round of 256 x 256
    tiles over the first 32,768 columns and the rest as one round of 256 x 144 tiles
    (the ops/gemm_tuning.json col_splits mechanism; not enabled for the step, where it measured no
    gain: profiles/r4_ab/lmhead_col_split.txt), against the fp32 reference and the unsplit launch."""
    M, N, K = 512, 50257, 768
    monkeypatch.setenv("DLS_COL_SPLIT", "1" if split else "0")
    ops.tuning.table()
    monkeypatch.setitem(ops.tuning._col_splits, ops.tuning._key(M, N, K), [(0, 32768, 13, 1), (32768, N, 42, 1)])
    x = _rand(M, K, scale=2.0, seed=210) + 0.3
    w = _rand(N, K, scale=0.05, seed=211)
    nw = (1 + 0.2 * _rand(K, seed=212).float()).to(torch.bfloat16)
    nb = _rand(K, scale=0.1, seed=213)
    xf = x.cpu().float()
    st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).to(DEV)
    wd, cs, bd = ops.derive_norm_gemm(w, nw, nb, None)
    ob = torch.full((1, M, 50304), float("nan"), device=DEV, dtype=torch.bfloat16)
    out = ob[:, :, :N]
    if split:
        assert ops.tuning.col_split(M, N, K) is not None
    ops.linear_norm(x.view(1, M, K), wd, cs, bd, "layernorm", out=out, ext_stats=st)
    torch.cuda.synchronize()
    ref = ops.ref_linear(ops.ref_layernorm(x.cpu(), nw.cpu(), nb.cpu()), w.cpu()).float()
    _close(out[0].cpu(), ref, 3e-2)
    assert torch.isnan(ob[:, :, N:].float()).all()  # the padding columns stay untouched


@pytest.mark.parametrize("pol", [1, 2, 3])
def test_lm_head_stream_policy(pol, monkeypatch):
    """The LM head with streaming (nt) cache policies (GemmArgs::stream_pol: bit 0 the weight
    DMA, bit 1 the logits stores; ops.LMHEAD_POL) computes exactly what the default policy
    does, and matches the fp32 reference."""
    M, N, K = 512, 50257, 768
    x = _rand(M, K, scale=2.0, seed=220) + 0.3
    w = _rand(N, K, scale=0.05, seed=221)
    nw = (1 + 0.2 * _rand(K, seed=222).float()).to(torch.bfloat16)
    nb = _rand(K, scale=0.1, seed=223)
    xf = x.cpu().float()
    st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).to(DEV)
    wd, cs, bd = ops.derive_norm_gemm(w, nw, nb, None)
    outs = {}
    for p_ in (0, pol):
        monkeypatch.setattr(ops, "LMHEAD_POL", p_)
        ob = torch.full((1, M, 50304), float("nan"), device=DEV, dtype=torch.bfloat16)
        ops.linear_norm(x.view(1, M, K), wd, cs, bd, "layernorm", out=ob[:, :, :N], ext_stats=st)
        torch.cuda.synchronize()
        assert torch.isnan(ob[:, :, N:].float()).all()
        outs[p_] = ob[0, :, :N].cpu()
    assert torch.equal(outs[0], outs[pol])
    ref = ops.ref_linear(ops.ref_layernorm(x.cpu(), nw.cpu(), nb.cpu()), w.cpu()).float()
    _close(outs[pol], ref, 3e-2)


@pytest.mark.parametrize("config", [12, 14, 17, 25, 27, 31, 38])
def test_gemm_stream_policy_plain(config):
    """stream_pol on plain GEMMs, split-ring and joint-ring configs incl. K groups (bias +
    residual epilogue): weight DMA nt, output stores nt or write-through — bit-identical to the
    default policy."""
    M, N, K = 384, 1024, 512
    x, w = _rand(M, K, seed=230), _rand(N, K, scale=0.05, seed=231)
    b, r = _rand(N, scale=0.1, seed=232), _rand(M, N, seed=233)
    e = ops.ext()
    ys = [e.gemm(x, w, b, r, 0, 1.0, None, config, 1, stream_pol=p_) for p_ in (0, 1, 2, 3, 4, 5)]
    torch.cuda.synchronize()
    for y in ys[1:]:
        assert torch.equal(ys[0], y)
    ref = ops.ref_linear(x.cpu(), w.cpu(), b.cpu()).float() + r.cpu().float()
    _close(ys[3].cpu(), ref, 2e-2)


@pytest.mark.parametrize("config,splitk,act", [(0, 2, 0), (0, 4, 0), (14, 4, 0), (12, 1, 4), (33, 1, 4)])
def test_gemm_write_through_splitk_swiglu(config, splitk, act):
    """Write-through stores (stream_pol bit 4) on split-K partial slabs + their reduce kernel and
    on the SwiGLU epilogue: bit-identical to the default stores."""
    M, N, K = 256, 1024, 1024
    x, w = _rand(M, K, seed=250), _rand(N, K, scale=0.05, seed=251)
    if act == 4:
        w = ops.interleave_gate_up(w)
    e = ops.ext()
    ys = [e.gemm(x, w, None, None, act, 1.0, None, config, splitk, stream_pol=p_) for p_ in (0, 4)]
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1])


def test_gemm_write_through_large_output():
    """A 2 GiB output keeps the default stores (policy stores address 32-bit buffer offsets):
    its last rows, past 2^31 bytes, must be written correctly under the write-through default."""
    M, N, K = 32768, 32768, 64
    x, w = _rand(M, K, seed=260), _rand(N, K, scale=0.05, seed=261)
    y = ops.ext().gemm(x, w, None, None, 0, 1.0, None, 0, 1, stream_pol=4)
    torch.cuda.synchronize()
    rows = torch.tensor([0, M // 2, M - 2, M - 1])
    ref = ops.ref_linear(x[rows.to(DEV)].cpu(), w.cpu()).float()
    _close(y[rows.to(DEV)].cpu(), ref, 2e-2)
    del y
    torch.cuda.empty_cache()


@pytest.mark.parametrize("S,n_head,n_kv,D", [(512, 12, 12, 64), (512, 32, 8, 128)])
def test_attention_write_through_stores(S, n_head, n_kv, D):
    """Attention flags (bit 0 write-through output stores, bit 1 XCD-grouped blocks) compute
    exactly what the default launch computes (batch 2: the grouping remaps batch and head)."""
    B = 2
    q = _rand(B * S, n_head * D, seed=240)
    k = _rand(B * S, n_kv * D, seed=241)
    v = _rand(B * S, n_kv * D, seed=242)
    e = ops.ext()
    o0 = e.attention(q, k, v, B, S, n_head, n_kv, D, True, 1.0 / D ** 0.5, None, 0, 0, 0, 0)
    for flags in (1, 2, 3):
        o1 = e.attention(q, k, v, B, S, n_head, n_kv, D, True, 1.0 / D ** 0.5, None, 0, 0, 0, flags)
        torch.cuda.synchronize()
        assert torch.equal(o0, o1), flags


def test_mlp_fused_one_launch():
    """The GPT-2 MLP block as ONE launch (gemm_fused.hip): folded LayerNorm-2 + fc1 + GELU, then
    fc2 + bias + residual + the next norm's row statistics, linked by in-launch arrival counters —
    against the fp32 reference, three launches in a row on one counter buffer (each launch resets
    its counters), no wait ever gave up."""
    M, H, F = 512, 768, 3072
    assert ops.mlp_fused_ok(M, H, F, H)
    x = _rand(M, H, scale=2.0, seed=300) + 0.2
    w1, b1 = _rand(F, H, scale=0.04, seed=301), _rand(F, scale=0.1, seed=302)
    w2, b2 = _rand(H, F, scale=0.02, seed=303), _rand(H, scale=0.1, seed=304)
    nw = (1 + 0.2 * _rand(H, seed=305).float()).to(torch.bfloat16)
    nb = _rand(H, scale=0.1, seed=306)
    res = _rand(M, H, seed=307)
    xf = x.cpu().float()
    st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).to(DEV)
    wd, cs, bd = ops.derive_norm_gemm(w1, nw, nb, b1)
    h = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    out = torch.empty(M, H, device=DEV, dtype=torch.bfloat16)
    sync = torch.zeros(2 * M // 64 + 1, dtype=torch.int32, device=DEV)
    for _ in range(3):
        so = torch.zeros(M, 2, device=DEV)
        ops.mlp_fused(x, wd, bd, cs, st, "layernorm", 1e-5, h, w2, b2, res, out, stats_out=so, sync=sync)
    torch.cuda.synchronize()
    hr = ops.ref_linear(ops.ref_layernorm(x.cpu(), nw.cpu(), nb.cpu()), w1.cpu(), b1.cpu(), act="gelu")
    ref = ops.ref_linear(hr, w2.cpu(), b2.cpu(), residual=res.cpu()).float()
    _close(h.cpu(), hr.float(), 3e-2)
    _close(out.cpu(), ref, 3e-2)
    of = out.cpu().float()
    _close(so.cpu(), torch.stack([of.sum(1), (of * of).sum(1)], 1), 1e-2)
    assert int(sync[-1]) == 0 and int(sync[:-1].abs().sum()) == 0  # no timeout; counters reset


@pytest.mark.parametrize("shared", [False, True])
def test_moe_xbatch_index_and_cross_request_experts(shared):
    """Cross-request expert batch (executor._run_moe_xbatch): the index launch maps groups
    (request, expert) onto their requests' expert-sorted blocks exactly as the host reference
    does, and ONE grouped gate/up + down pair over those groups — the same expert weights in
    several groups, run panel-major with cached weights when ``shared`` — equals each request's
    expert computed alone in fp32."""
    Q, M, E, k, H, F = 3, 200, 8, 2, 256, 384
    g = torch.Generator().manual_seed(17)
    routes, xs = [], []
    for q in range(Q):
        logits = torch.randn(M, E, generator=g).to(torch.bfloat16).to(DEV)
        routes.append(ops.moe_route(logits, k, E))
        xs.append(_rand(M, H, seed=60 + q))
    R = M * k
    pairs = [(0, 1), (1, 1), (2, 1), (0, 5), (2, 5), (1, 6)]  # (request, expert); expert 1 in three groups
    reqs, experts = [q for q, _ in pairs], [e for _, e in pairs]
    offsets = torch.zeros(len(pairs) + 1, dtype=torch.int32, device=DEV)
    a_rows = torch.full((Q * R,), -1, dtype=torch.int32, device=DEV)
    ops.moe_xbatch_index([r[4] for r in routes], reqs, experts, [q * R for q in range(Q)], offsets, a_rows)
    o_ref, a_ref = torch.zeros(len(pairs) + 1, dtype=torch.int32), torch.zeros(Q * R, dtype=torch.int32)
    ops.moe_xbatch_index([r[4].cpu() for r in routes], reqs, experts, [q * R for q in range(Q)], o_ref, a_ref)
    torch.cuda.synchronize()
    assert offsets.cpu().tolist() == o_ref.tolist()
    n = int(o_ref[-1])
    assert a_rows[:n].cpu().tolist() == a_ref[:n].tolist()
    # the batch: each request's rows in its block of one token matrix
    xp = torch.cat([ops.moe_permute(xs[q], routes[q][2]) for q in range(Q)])
    w13 = {e: ops.interleave_gate_up(_rand(2 * F, H, scale=0.05, seed=80 + e)) for e in set(experts)}
    w2 = {e: _rand(H, F, scale=0.05, seed=90 + e) for e in set(experts)}
    h = torch.full((Q * R, F), 3.0, dtype=torch.bfloat16, device=DEV)
    outs = [torch.full((M, H), 7.0, dtype=torch.bfloat16, device=DEV) for _ in pairs]
    ops.gemm_grouped(xp, [w13[e] for e in experts], offsets, act="swiglu", out=h, rows_hint=R // E, a_rows=a_rows,
                     shared_weights=shared)
    ops.gemm_grouped(h, [w2[e] for e in experts], offsets, outs=outs, rows_hint=R // E, shared_weights=shared)
    torch.cuda.synchronize()
    for gi, (q, e) in enumerate(pairs):
        off = routes[q][4].cpu().tolist()
        rows = routes[q][2].cpu()[off[e]:off[e + 1]].long()
        cnt = rows.numel()
        ref = ops.ref_linear(ops.ref_linear(xs[q].cpu()[rows], w13[e].cpu(), act="swiglu").to(torch.bfloat16),
                             w2[e].cpu())
        _close(outs[gi][:cnt].cpu(), ref.float(), 3e-2)
        assert (outs[gi][cnt:].cpu().float() == 7.0).all(), "rows past the group's count were written"


@pytest.mark.parametrize("B,S,H,nh", [(1, 512, 768, 12), (2, 256, 768, 12), (4, 128, 768, 12), (1, 1024, 768, 12),
                                      (1, 512, 1024, 16)])
def test_attn_block_one_launch(B, S, H, nh):
    """The pre-norm attention block as ONE launch (attn_block.hip): folded LayerNorm-1 + QKV GEMM,
    causal MHA, out-proj + bias + residual + the next norm's row statistics, linked by in-launch
    ticket-ordered items and arrival counters — against the fp32 reference (GPT-2's block at
    batch 1 x 512 and smaller shapes), three launches in a row on one counter buffer (each
    resets its counters), no wait ever gave up."""
    M, D = B * S, H // nh
    assert ops.attn_block_ok(M, H, B, S, nh, nh, D)
    x = _rand(M, H, scale=2.0, seed=400) + 0.2
    w1, b1 = _rand(3 * H, H, scale=0.04, seed=401), _rand(3 * H, scale=0.1, seed=402)
    wo, bo = _rand(H, H, scale=0.03, seed=403), _rand(H, scale=0.1, seed=404)
    nw = (1 + 0.2 * _rand(H, seed=405).float()).to(torch.bfloat16)
    nb = _rand(H, scale=0.1, seed=406)
    res = _rand(M, H, seed=407)
    xf = x.cpu().float()
    st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).to(DEV)
    wd, cs, bd = ops.derive_norm_gemm(w1, nw, nb, b1)
    qkv = torch.empty(M, 3 * H, device=DEV, dtype=torch.bfloat16)
    o = torch.empty(M, H, device=DEV, dtype=torch.bfloat16)
    out = torch.empty(M, H, device=DEV, dtype=torch.bfloat16)
    sync = ops.attn_block_sync(M, S, B, nh, DEV)
    for _ in range(3):
        so = torch.zeros(M, 2, device=DEV)
        ops.attn_block(x, wd, bd, cs, st, "layernorm", 1e-5, qkv, o, wo, bo, res, out, B, S, nh, stats_out=so,
                       sync=sync)
    torch.cuda.synchronize()
    qr = ops.ref_linear(ops.ref_layernorm(x.cpu(), nw.cpu(), nb.cpu()), w1.cpu(), b1.cpu())
    orf = ops.ref_attention(qr[:, :H], qr[:, H:2 * H], qr[:, 2 * H:], B, S, nh, nh, D, causal=True)
    ref = ops.ref_linear(orf, wo.cpu(), bo.cpu(), residual=res.cpu()).float()
    _close(qkv.cpu(), qr.float(), 3e-2)
    _close(o.cpu(), orf.float(), 3e-2)
    _close(out.cpu(), ref, 3e-2)
    of = out.cpu().float()
    _close(so.cpu(), torch.stack([of.sum(1), (of * of).sum(1)], 1), 1e-2)
    assert int(sync[-1]) == 0 and int(sync[:-1].abs().sum()) == 0  # no timeout; counters reset


def test_attn_block_shape_gate():
    """Shapes the one-launch block does not take fall back to the three launches (executor)."""
    assert ops.attn_block_ok(512, 768, 1, 512, 12, 12, 64)
    assert ops.attn_block_ok(512, 1024, 1, 512, 16, 16, 64)       # GPT-2-medium
    assert not ops.attn_block_ok(512, 4096, 1, 512, 32, 8, 128)   # Llama: GQA, head_dim 128
    assert not ops.attn_block_ok(480, 768, 1, 480, 12, 12, 64)    # rows not a multiple of 64
