#!/usr/bin/env python3
"""Per-kernel microbenchmarks on MI355X: our HIP kernels vs torch's library paths
(hipBLASLt GEMM via torch.matmul, SDPA, F.layer_norm) on the DAG's real shapes.

Timing: hipEvents around N back-to-back launches after warmup, median of 5 rounds,
random operands (never zero-filled — cdna_hip_programming.md §5.4 rule 25). Every
variant is interleaved in one process (rule 24). Prints one JSON line per case.

    python benchmarks/bench_kernels.py [--quick] [--only gemm|attn|norm]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402

DEV = "cuda"


def timeit(fn, iters=20, rounds=5):
    """Median device time per call (us): ``iters`` calls captured in one hipGraph, so
    host launch overhead does not mask the kernel time (ours and torch's alike)."""
    from distributed_llm_scheduler_amd.ops.tuning import _graph_time
    return _graph_time(lambda i: fn(), reps=iters, rounds=rounds)


GEMMS = [  # (label, M, N, K)
    ("gpt2.qkv", 512, 2304, 768), ("gpt2.proj", 512, 768, 768), ("gpt2.fc1", 512, 3072, 768),
    ("gpt2.fc2", 512, 768, 3072), ("gpt2.lm_head", 512, 50257, 768),
    ("llama8b.qkv", 512, 6144, 4096), ("llama8b.wo", 512, 4096, 4096), ("llama8b.w13", 512, 28672, 4096),
    ("llama8b.w2", 512, 4096, 14336), ("sq4096", 4096, 4096, 4096),
]


def bench_gemm(quick):
    ext = ops.ext()
    for label, M, N, K in (GEMMS[:5] if quick else GEMMS):
        x = (torch.randn(M, K, device=DEV) * 0.5).bfloat16()
        w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        t_torch = timeit(lambda: torch.matmul(x, w.t(), out=out))
        row = {"kind": "gemm", "case": label, "M": M, "N": N, "K": K, "torch_us": round(t_torch, 2),
               "torch_tflops": round(flops / t_torch / 1e6, 1)}
        t_auto = timeit(lambda: ext.gemm(x, w, None, None, 0, 1.0, out, -1, 0))
        row["auto"] = list(ext.gemm_glds_pick(M, N, K))
        row["auto_us"] = round(t_auto, 2)
        row["auto_tflops"] = round(flops / t_auto / 1e6, 1)
        t_old = timeit(lambda: ext.gemm(x, w, None, None, 0, 1.0, out, ext.REGSTAGE + ext.gemm_pick_config(M, N, K), 1))
        row["regstage_us"] = round(t_old, 2)
        best = None
        for cfg in range(ext.gemm_glds_num_configs()):
            for sk in (1, 2, 3, 4, 6, 8):
                if K % (64 * sk) or (sk > 1 and N % 8):
                    continue
                if sk > 1 and M * N > 4096 * 4096:
                    continue
                t = timeit(lambda: ext.gemm(x, w, None, None, 0, 1.0, out, cfg, sk), iters=10, rounds=3)
                row[f"c{cfg}s{sk}"] = round(t, 2)
                if best is None or t < best[1]:
                    best = ((cfg, sk), t)
        row["best"], row["best_us"] = best[0], round(best[1], 2)
        row["best_tflops"] = round(flops / best[1] / 1e6, 1)
        from distributed_llm_scheduler_amd.ops import tuning
        cold, _ = tuning.tune(M, N, K, save=True)
        row["cold_tuned"], row["cold_tuned_us"] = cold[:2], round(cold[2], 2)
        print(json.dumps(row), flush=True)


def bench_attn(quick):
    cases = [("gpt2", 1, 512, 12, 12, 64), ("llama8b", 1, 512, 32, 8, 128), ("gpt2.b8", 8, 512, 12, 12, 64),
             ("llama8b.s2k", 1, 2048, 32, 8, 128)]
    for label, B, S, nh, nkv, D in (cases[:2] if quick else cases):
        qkv = torch.randn(B * S, (nh + 2 * nkv) * D, device=DEV).bfloat16()
        q, k, v = qkv[:, :nh * D], qkv[:, nh * D:(nh + nkv) * D], qkv[:, (nh + nkv) * D:]
        o = torch.empty(B * S, nh * D, device=DEV, dtype=torch.bfloat16)
        ours = timeit(lambda: ops.attention(q, k, v, B, S, nh, nkv, D, True, out=o))
        sc = 1.0 / math.sqrt(D)
        var = {f"v{vv}": round(timeit(lambda: ops.ext().attention(q, k, v, B, S, nh, nkv, D, True, sc, o, vv)), 2)
               for vv in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13)}
        qh = q.reshape(B, S, nh, D).transpose(1, 2).contiguous()
        kh = k.reshape(B, S, nkv, D).transpose(1, 2).repeat_interleave(nh // nkv, 1).contiguous()
        vh = v.reshape(B, S, nkv, D).transpose(1, 2).repeat_interleave(nh // nkv, 1).contiguous()
        ref = timeit(lambda: F.scaled_dot_product_attention(qh, kh, vh, is_causal=True))
        flops = 2.0 * 2 * B * nh * S * S * D / 2
        print(json.dumps({"kind": "attn", "case": label, "ours_us": round(ours, 2), "torch_sdpa_us": round(ref, 2),
                          "ours_tflops": round(flops / ours / 1e6, 1), **var}), flush=True)


def bench_norm(quick):
    for M, H in ((512, 768), (512, 4096), (4096, 4096)):
        x = torch.randn(M, H, device=DEV).bfloat16()
        r = torch.randn(M, H, device=DEV).bfloat16()
        w, b = torch.ones(H, device=DEV).bfloat16(), torch.zeros(H, device=DEV).bfloat16()
        y = torch.empty_like(x)
        ours = timeit(lambda: ops.layernorm(x, w, b, out=y))
        fused = timeit(lambda: ops.layernorm(x, w, b, residual=r, out=y))
        ref = timeit(lambda: F.layer_norm(x, (H,), w, b))
        gb = 2 * M * H * 2 / 1e9
        rms = timeit(lambda: ops.rmsnorm(x, w, out=y))
        print(json.dumps({"kind": "layernorm", "M": M, "H": H, "ours_us": round(ours, 2),
                          "ours_add_ln_us": round(fused, 2), "ours_rms_us": round(rms, 2), "torch_us": round(ref, 2),
                          "ours_GBps": round(gb / ours * 1e6, 1)}), flush=True)
    S, nh, nkv, D = 512, 32, 8, 128
    qkv = torch.randn(S, (nh + 2 * nkv) * D, device=DEV).bfloat16()
    cos, sin = ops.rope_tables(S, D, 500000.0, DEV)
    t = timeit(lambda: ops.rope_(qkv, S, nh, nkv, D, nh * D, cos, sin))
    print(json.dumps({"kind": "rope", "M": S, "heads": nh + nkv, "D": D, "ours_us": round(t, 2)}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    if a.only in ("", "gemm"):
        bench_gemm(a.quick)
    if a.only in ("", "attn"):
        bench_attn(a.quick)
    if a.only in ("", "norm"):
        bench_norm(a.quick)
