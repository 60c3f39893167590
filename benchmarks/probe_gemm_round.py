#!/usr/bin/env python3
"""One round (exactly 256 tiles) of a GEMM config on the LM-head K, launched eagerly N times —
a short target for rocprofv3 --pmc passes (per-dispatch counters of one kernel shape). Prints
the mean device time per launch (hipEvents).

    --hot      A and W rows alias one 256-row block (row stride 0 beyond it is not allowed, so
               the operands are as_strided views over ONE row each): every DMA hits L2 —
               the kernel's ceiling with no memory system in the way
    --rotate R cycle R weight copies (cold weights, as in the DAG step)

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... --kernel-trace -d out -- python3 benchmarks/probe_gemm_round.py --cfg 34
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", type=int, default=34)
ap.add_argument("--bm", type=int, default=256)
ap.add_argument("--bn", type=int, default=256)
ap.add_argument("--M", type=int, default=512)
ap.add_argument("--K", type=int, default=768)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--rotate", type=int, default=1)
ap.add_argument("--hot", action="store_true")
ap.add_argument("--zeros", action="store_true", help="zero operands (DVFS comparison)")
ap.add_argument("--ldpad", type=int, default=0, help="extra output row stride (elements)")
a = ap.parse_args()
ext = ops.ext()
N = 256 * a.bm * a.bn // a.M
mk = (lambda *s: torch.zeros(*s, device="cuda", dtype=torch.bfloat16)) if a.zeros else \
    (lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16())
if a.hot:
    xr, wr = mk(1, a.K), mk(1, a.K)
    x = xr.as_strided((a.M, a.K), (0, 1))
    ws = [wr.as_strided((N, a.K), (0, 1))]
else:
    x = mk(a.M, a.K)
    ws = [mk(N, a.K) for _ in range(a.rotate)]
o = torch.empty(a.M, N + a.ldpad, device="cuda", dtype=torch.bfloat16)[:, :N]
for i in range(3):
    ext.gemm(x, ws[i % len(ws)], None, None, 0, 1.0, o, a.cfg, 1)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for i in range(a.reps):
    ext.gemm(x, ws[i % len(ws)], None, None, 0, 1.0, o, a.cfg, 1)
ev[1].record()
torch.cuda.synchronize()
us = ev[0].elapsed_time(ev[1]) * 1e3 / a.reps
fl = 2.0 * a.M * N * a.K
src = torch.empty(a.M, N, device="cuda", dtype=torch.bfloat16)
ev[0].record()
for i in range(a.reps):
    o.copy_(src)
ev[1].record()
torch.cuda.synchronize()
cu = ev[0].elapsed_time(ev[1]) * 1e3 / a.reps
print(f"cfg {a.cfg} N {N} ldpad {a.ldpad} hot={a.hot} rotate={a.rotate}: {us:.2f} us/launch, {fl / us / 1e6:.0f} TFLOP/s; torch copy of the output {cu:.2f} us", flush=True)
