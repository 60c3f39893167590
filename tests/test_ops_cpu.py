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
