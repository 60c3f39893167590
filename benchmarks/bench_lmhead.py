#!/usr/bin/env python3
"""LM-head GEMM (GPT-2: out[512, 50257] = x[512, 768] @ wte^T) on MI355X: every LDS-DMA config
(plain and persistent) against the vendor library, plus a ONE-ROUND probe (exactly 256 tiles of
the config on 256 CUs) that gives the per-tile time — the LM head's 394 / 786 tiles quantise
into rounds, so per-tile time x rounds is what a config can reach.

    python benchmarks/bench_lmhead.py [--cfgs 0,8,12,13,14] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops.tuning import PERSIST, _graph_time  # noqa: E402

SHAPES = {36: (256, 224), 0: (256, 128), 1: (128, 128), 8: (256, 256), 9: (256, 256), 12: (256, 256), 13: (256, 256),
          14: (256, 128), 7: (128, 128), 15: (128, 128), 10: (256, 128), 34: (256, 256), 35: (256, 256)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="34,35,8,10")
    ap.add_argument("--M", type=int, default=512)
    ap.add_argument("--N", type=int, default=50257)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ext = ops.ext()
    torch.manual_seed(0)
    M, N, K = a.M, a.N, a.K
    ldo = (N + 63) // 64 * 64
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    # several weight copies, rotated per call: cold-ish weights as in the DAG step (77 MB each)
    ws = [(torch.rand(N, K, device="cuda") * 2 - 1).bfloat16() for _ in range(4)]
    ob = torch.empty(M, ldo, device="cuda", dtype=torch.bfloat16)
    o = ob[:, :N]
    res = []
    flops = 2.0 * M * N * K

    def rec(name, us, extra=None):
        r = {"cfg": name, "us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}
        if extra:
            r.update(extra)
        res.append(r)
        print(json.dumps(r), flush=True)

    rec("torch", _graph_time(lambda i: torch.matmul(x, ws[i % 4].t(), out=o), reps=8))
    ref = (x.float() @ ws[0].float().t())
    for c in [int(v) for v in a.cfgs.split(",")]:
        for persist in ((0,) if c >= 34 else (0, PERSIST)):
            cfg = c + persist
            try:
                ext.gemm(x, ws[0], None, None, 0, 1.0, o, cfg, 1)
                torch.cuda.synchronize()
                err = (o.float() - ref).abs().max().item()
                us = _graph_time(lambda i: ext.gemm(x, ws[i % 4], None, None, 0, 1.0, o, cfg, 1), reps=8)
            except RuntimeError as e:
                print(json.dumps({"cfg": cfg, "error": str(e)[:200]}), flush=True)
                continue
            extra = {"err": round(err, 3)}
            bm, bn = SHAPES.get(c, (0, 0))
            if bm and not persist:
                # one round: exactly 256 tiles of this config
                n1 = 256 * bm * bn // M
                w1 = ws[0][:n1]
                o1 = torch.empty(M, n1, device="cuda", dtype=torch.bfloat16)
                extra["one_round_us"] = round(_graph_time(lambda i: ext.gemm(x, ws[i % 4][:n1], None, None, 0, 1.0,
                                                                             o1, cfg, 1), reps=8), 2)
                extra["tiles"] = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
                del w1
            rec(cfg, us, extra)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
