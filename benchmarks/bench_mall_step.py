#!/usr/bin/env python3
"""Does the once-per-step LM-head traffic (77 MB weight read + 51 MB logits written) push GPT-2's
170 MB of layer weights out of the 256 MB Infinity Cache? A synthetic GPT-2 step (12 x the four
layer GEMMs with their tuned configs, then the LM head) in one hipGraph, with the LM-head
weight and/or the logits in normal or uncached (hipDeviceMallocUncached) device memory."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402
from distributed_llm_scheduler_amd.ops import tuning  # noqa: E402


def timed_graph(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    e = ops.ext()
    M, H, F, V = 512, 768, 3072, 50257
    shapes = [(3 * H, H), (H, H), (F, H), (H, F)]
    layers = [[(torch.randn(n, k, device="cuda") * 0.05).bfloat16() for n, k in shapes] for _ in range(12)]
    cfgs = [tuning.lookup(M, n, k) for n, k in shapes]
    x = (torch.randn(M, H, device="cuda") * 0.5).bfloat16()
    xf = (torch.randn(M, F, device="cuda") * 0.5).bfloat16()
    outs = [torch.empty(M, n, device="cuda", dtype=torch.bfloat16) for n, _ in shapes]

    def gemm(a, w, out, cfg):
        c, sk = cfg
        if c >= tuning.REGSTAGE or c == tuning.LIB:
            torch.mm(a, w.t(), out=out)
        else:
            e.gemm(a, w, None, None, 0, 1.0, out, c, sk)

    res = {}
    for wte_unc in (False, True):
        for log_unc in (False, True):
            wte = (e.alloc_device(V * H * 2, 3).view(torch.bfloat16).view(V, H) if wte_unc
                   else torch.empty(V, H, device="cuda", dtype=torch.bfloat16))
            wte.copy_((torch.randn(V, H, device="cuda") * 0.05).bfloat16())
            logits = (e.alloc_device(M * V * 2, 3).view(torch.bfloat16).view(M, V) if log_unc
                      else torch.empty(M, V, device="cuda", dtype=torch.bfloat16))

            def layers_only():
                for ws in layers:
                    gemm(x, ws[0], outs[0], cfgs[0])
                    gemm(x, ws[1], outs[1], cfgs[1])
                    gemm(x, ws[2], outs[2], cfgs[2])
                    gemm(xf, ws[3], outs[3], cfgs[3])

            def step():
                layers_only()
                torch.mm(x, wte.t(), out=logits)

            key = f"wte_{'unc' if wte_unc else 'cached'}_logits_{'unc' if log_unc else 'cached'}"
            res[key + "_step_us"] = round(timed_graph(step), 1)
            res[key + "_lmhead_us"] = round(timed_graph(lambda: torch.mm(x, wte.t(), out=logits)), 1)
            if not wte_unc and not log_unc:
                res["layers_only_us"] = round(timed_graph(layers_only), 1)
            del wte, logits
            torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
