"""CPU semantics of op-level helpers shared by the GPU path (layouts, ranged GEMM)."""
import torch

from distributed_llm_scheduler_amd import ops


def test_interleave_gate_up_layout_and_swiglu():
    F, K = 48, 8
    w = torch.arange(2 * F * K, dtype=torch.float32).reshape(2 * F, K)
    wi = ops.interleave_gate_up(w)
    assert torch.equal(wi[0:16], w[0:16]) and torch.equal(wi[16:32], w[F:F + 16])
    assert torch.equal(wi[32:48], w[16:32]) and torch.equal(wi[80:96], w[F + 32:F + 48])
    x = torch.randn(5, K)
    y = ops.ref_linear(x, wi, act="swiglu")
    full = x @ w.t()
    assert torch.allclose(y, torch.nn.functional.silu(full[:, :F]) * full[:, F:], atol=1e-4)
    b = torch.randn(2 * F)
    assert torch.equal(ops.interleave_gate_up(b)[16:32], b[F:F + 16])


def test_ranged_linear_cpu_only_touches_range():
    x, w = torch.randn(10, 16), torch.randn(8, 16)
    out = torch.full((10, 8), 7.0)
    ops.linear(x, w, out=out, rows=torch.tensor([3, 6], dtype=torch.int32))
    assert (out[:3] == 7).all() and (out[6:] == 7).all()
    assert torch.allclose(out[3:6], x[3:6] @ w.t(), atol=1e-5)


def test_moe_route_and_gathered_grouped_gemm_cpu():
    """CPU fallbacks: moe_route == moe_router + moe_align, and a grouped GEMM reading its
    expert-sorted rows through a_rows equals the permute-then-GEMM path."""
    M, E, k, H, F = 40, 4, 2, 16, 8
    g = torch.Generator().manual_seed(3)
    logits = torch.stack([torch.randperm(E, generator=g) for _ in range(M)]).float().to(torch.bfloat16)
    idx, gate, src, slot, off = ops.moe_route(logits, k, E)
    ri, rg = ops.moe_router(logits, k)
    rs, rsl, ro = ops.moe_align(ri, E)
    assert torch.equal(idx, ri) and torch.equal(gate, rg)
    assert torch.equal(src, rs) and torch.equal(slot, rsl) and torch.equal(off, ro)
    x = torch.randn(M, H, generator=g).to(torch.bfloat16)
    ws = [(torch.randn(F, H, generator=g) * 0.1).to(torch.bfloat16) for _ in range(E)]
    R = src.numel()
    a = ops.gemm_grouped(ops.moe_permute(x, src), ws, off, out=torch.zeros(R, F, dtype=torch.bfloat16))
    b = ops.gemm_grouped(x, ws, off, out=torch.zeros(R, F, dtype=torch.bfloat16), a_rows=src)
    assert torch.equal(a, b)


def test_tuning_model_overrides(tmp_path, monkeypatch):
    """A model's own choice for a GEMM shape it shares with other models (tuning
    ``model_overrides``) wins while that model's executor runs, and in-DAG refinement of that
    shape updates the override, not the shared entry."""
    import json

    from distributed_llm_scheduler_amd.ops import tuning

    path = tmp_path / "t.json"
    path.write_text(json.dumps({"gemm": {"512x6144x4096": [38, 1]}, "candidates": {}, "refined": {},
                                "model_overrides": {"mixtral-8x7b": {"512x6144x4096": [0, 2]}}}))
    monkeypatch.setattr(tuning, "_PATH", str(path))
    monkeypatch.setattr(tuning, "_table", None)
    monkeypatch.setattr(tuning, "_overrides", {})
    monkeypatch.setattr(tuning, "_cands", {})
    monkeypatch.setattr(tuning, "_refined", {})
    monkeypatch.setattr(tuning, "_model", None)
    assert tuning.lookup(512, 6144, 4096) == (38, 1)
    tuning.set_model("mixtral-8x7b")
    assert tuning.lookup(512, 6144, 4096) == (0, 2)
    tuning.set_choice(512, 6144, 4096, "", (14, 4))
    assert tuning.lookup(512, 6144, 4096) == (14, 4)
    tuning.set_model("llama3-8b")
    assert tuning.lookup(512, 6144, 4096) == (38, 1)
    tuning.save()
    doc = json.loads(path.read_text())
    assert doc["gemm"]["512x6144x4096"] == [38, 1]
    assert doc["model_overrides"]["mixtral-8x7b"]["512x6144x4096"] == [14, 4]


def test_stream_policy_selection(monkeypatch):
    """Cache policy per GEMM (ops._stream_pol): vocabulary-sized projections (the LM head) get
    the LM-head policy, every other GEMM the activation policy, plus weight-nt above the size
    threshold when one is set."""
    from distributed_llm_scheduler_amd import ops
    monkeypatch.setattr(ops, "LMHEAD_POL", 3)
    monkeypatch.setattr(ops, "ACT_POL", 4)
    monkeypatch.setattr(ops, "WEIGHT_NT_MB", 0.0)
    monkeypatch.setattr(ops, "_ACT_POL_SET", False)
    monkeypatch.setattr(ops.tuning, "_model", None)
    assert ops._stream_pol(50257, 768) == 3      # GPT-2's 77 MB LM head
    assert ops._stream_pol(128256, 4096) == 4    # Llama-3's 1 GB LM head: an ordinary GEMM
    assert ops._stream_pol(2304, 768) == 4
    monkeypatch.setattr(ops, "WEIGHT_NT_MB", 20.0)
    assert ops._stream_pol(28672, 4096) == 5  # 235 MB gate/up weight: nt DMA + write-through
    assert ops._stream_pol(2304, 768) == 4    # 3.5 MB: below the threshold
    monkeypatch.setattr(ops, "WEIGHT_NT_MB", 0.0)
    # per-model output-store default (Mixtral measured faster with default-policy stores) ...
    monkeypatch.setattr(ops.tuning, "_model", "mixtral-8x7b")
    assert ops._stream_pol(6144, 4096) == 0
    monkeypatch.setattr(ops.tuning, "_model", "llama3-8b")
    assert ops._stream_pol(6144, 4096) == 4
    # ... which an explicit DLS_ACT_POL overrides
    monkeypatch.setattr(ops, "_ACT_POL_SET", True)
    monkeypatch.setattr(ops.tuning, "_model", "mixtral-8x7b")
    assert ops._stream_pol(6144, 4096) == 4


def test_gemm_config_tables_agree():
    """The Python tuner's view of the LDS-DMA GEMM configs (K step per config, SwiGLU-unsafe
    configs) matches the kernel library's tables in csrc/kernels/gemm_glds.hip."""
    import os
    import re
    from distributed_llm_scheduler_amd.ops import tuning
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "csrc", "kernels", "gemm_glds.hip")).read()
    kstep = [int(v) for v in re.search(r"kKStep\[\] = \{([^}]*)\}", src).group(1).replace("\n", " ").split(",")]
    ncfg = int(re.search(r"constexpr int kNumCfg = (\d+);", src).group(1))
    assert len(kstep) == ncfg == len(tuning._KSTEP)
    assert kstep == list(tuning._KSTEP)
    bad = re.search(r"constexpr bool swiglu_bad\(int c\) \{ return ([^;]*); \}", src).group(1)
    lib_bad = {c for c in range(ncfg) if eval(bad.replace("&&", " and ").replace("||", " or "), {"c": c})}
    assert lib_bad == set(tuning.SWIGLU_BAD)


def test_no_tuning_entry_resolves_to_the_vendor_library_by_default():
    """Every GEMM the table knows runs on the hand-written kernels unless DLS_ALLOW_VENDOR_GEMM=1:
    no entry (plain, variant, per-model override, runner-up) resolves to hipBLASLt."""
    from distributed_llm_scheduler_amd.ops import tuning

    assert not tuning.VENDOR
    t = tuning.table()
    assert t, "tuning table missing"
    for key in t:
        shape, tg = key, ""
        while shape[-1].isalpha():
            shape, tg = shape[:-1], shape[-1] + tg
        M, N, K = (int(v) for v in shape.split("x"))
        assert tuning.lookup(M, N, K, tg)[0] != tuning.LIB, key
        assert all(c[0] != tuning.LIB for c in tuning.runner_ups(M, N, K, tg, 10)), key
        for m in tuning._overrides:
            tuning.set_model(m)
            assert tuning.lookup(M, N, K, tg)[0] != tuning.LIB, (m, key)
        tuning.set_model(None)
        assert (tuning.LIB, 1) not in tuning.candidates(M, N, K, 48, tg)
