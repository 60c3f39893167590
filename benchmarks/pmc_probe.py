#!/usr/bin/env python3
"""The program to put after ``--`` in a ``rocprofv3 --pmc`` pass (scripts/gpu.sh pmc): a few
launches of one hot GEMM exactly as the DAG step issues it, with cold weights (rotated
copies larger than the MALL where the step's weights are), so per-dispatch hardware counters
can name what bounds it (tools/pmc_summary.py).

    python benchmarks/pmc_probe.py lmhead        GPT-2 LM head: 512 x 50257 x 768, tuned config,
                                                 final LayerNorm folded (external row statistics)
    python benchmarks/pmc_probe.py moe           Mixtral-8x7B layer: the grouped gate/up (SwiGLU)
                                                 and down launches over 8 experts, 512 tokens top-2
    python benchmarks/pmc_probe.py gemm M N K    any plain GEMM shape with its tuned config
    python benchmarks/pmc_probe.py attn          GPT-2 causal attention: S 512, 12 heads x 64, the
                                                 launcher's variant
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402

REPS = int(os.environ.get("PMC_REPS", "4"))


def lmhead():
    M, N, K = 512, 50257, 768
    ldo = (N + 63) // 64 * 64
    x = (torch.randn(M, K, device="cuda") * 2).bfloat16()
    ws = [(torch.randn(N, K, device="cuda") * 0.05).bfloat16() for _ in range(4)]  # 4 x 77 MB: MALL-cold
    cs = ws[0].float().sum(1).contiguous()
    xf = x.float()
    st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).contiguous()
    ob = torch.empty(M, ldo, device="cuda", dtype=torch.bfloat16)
    cfg, sk = tuning.lookup_fused(M, N, K)
    print(f"lmhead cfg {cfg} splitk {sk}", flush=True)
    for i in range(REPS):
        ops.ext().gemm(x, ws[i % 4], None, None, 0, 1.0, ob[:, :N], cfg, sk, cs, 1, 1e-5, None, False, None, None, 1, 2,
                       0, None, st)
    torch.cuda.synchronize()


def moe(cfg_gateup=None, cfg_down=None):
    """``moe [gate/up config] [down config]``: the table's tiles, or the named configs (to
    compare e.g. the two-workgroups-per-CU tiles 46 / 47 against the table's)."""
    E, T, k, H, F = 8, 512, 2, 4096, 14336
    R = T * k
    if cfg_gateup is not None:
        tuning.set_choice(R // E, 2 * F, H, "sg", (int(cfg_gateup), 1))
    if cfg_down is not None:
        tuning.set_choice(R // E, H, F, "g", (int(cfg_down), 1))
    print("moe gate/up cfg", tuning.lookup_fused(R // E, 2 * F, H, "sg")[0], "down cfg",
          tuning.lookup_fused(R // E, H, F, "g")[0], flush=True)
    g = torch.Generator().manual_seed(7)
    cnt = torch.bincount(torch.randint(0, E, (R,), generator=g), minlength=E)
    off = torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0)]).to(torch.int32).cuda()
    rows = torch.randint(0, T, (R,), generator=g).to(torch.int32).cuda()
    x = (torch.randn(T, H, device="cuda") * 0.5).bfloat16()
    w13 = [(torch.randn(2 * F, H, device="cuda") * 0.02).bfloat16() for _ in range(E)]  # 1.9 GB
    w2 = [(torch.randn(H, F, device="cuda") * 0.02).bfloat16() for _ in range(E)]       # 0.94 GB
    h = torch.empty(R, F, device="cuda", dtype=torch.bfloat16)
    outs = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(E)]
    for _ in range(REPS):
        ops.gemm_grouped(x, w13, off, act="swiglu", out=h, rows_hint=R // E, a_rows=rows)
        ops.gemm_grouped(h, w2, off, outs=outs, rows_hint=R // E)
    torch.cuda.synchronize()


def attn():
    S, Hh, D = 512, 12, 64
    qkv = (torch.randn(S, 3 * Hh * D, device="cuda") * 0.5).bfloat16()
    q, k, v = qkv[:, :Hh * D], qkv[:, Hh * D:2 * Hh * D], qkv[:, 2 * Hh * D:]
    o = torch.empty(S, Hh * D, device="cuda", dtype=torch.bfloat16)
    for _ in range(REPS):
        ops.attention(q, k, v, 1, S, Hh, Hh, D, causal=True, out=o)
    torch.cuda.synchronize()


def gemm(M, N, K):
    x = (torch.randn(M, K, device="cuda")).bfloat16()
    ws = [(torch.randn(N, K, device="cuda") * 0.05).bfloat16() for _ in range(4)]
    cfg, sk = tuning.lookup(M, N, K)
    print(f"gemm {M}x{N}x{K} cfg {cfg} splitk {sk}", flush=True)
    for i in range(REPS):
        ops.linear(x, ws[i % 4])
    torch.cuda.synchronize()


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "lmhead":
        lmhead()
    elif what == "moe":
        moe(*sys.argv[2:4])
    elif what == "attn":
        attn()
    else:
        gemm(*(int(v) for v in sys.argv[2:5]))
