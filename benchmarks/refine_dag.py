#!/usr/bin/env python3
"""Exhaustive in-DAG GEMM config refinement: every valid (config, split-K) of each GEMM shape
of the model's step is timed inside the captured hipGraph of the REAL step (coordinate descent,
costliest shape first) and the fastest kept. Writes the table named by DLS_GEMM_TUNING.

    DLS_GEMM_TUNING=gpurun_out/t.json python benchmarks/refine_dag.py --model gpt2
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--batch", type=int, default=1, help="batch of the one request (8: bench.py's merged strong run)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=1, help="coordinate-descent passes over the shapes")
    ap.add_argument("--cfgs", default=None, help="only candidates with these config ids (comma list)")
    ap.add_argument("--keys", default=None, help="only these shape keys, e.g. 512x50257x768 (comma list)")
    ap.add_argument("--min-gain", type=float, default=0.002)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    plan = runtime.plan(args.model, world=1, seq=args.seq, batch=args.batch)
    store = runtime.make_store(plan, device_init=True)
    ex = runtime.make_executor(plan, 0, dev, store)
    for _ in range(3):
        ex.step()
    torch.cuda.synchronize()
    assert ex.capture()
    timings = []

    def log(key, cand, ms):
        timings.append((key, list(cand), round(ms, 5)))
        print(f"  {key} {cand}: {ms:.4f} ms", file=sys.stderr, flush=True)

    out = {}
    for r in range(args.rounds):
        out[f"round{r}"] = {k: [list(v[0]), list(v[1]), v[2]] for k, v in
                            ex.refine_tuning(reps=args.reps, min_gain=args.min_gain, force=True, exhaustive=True, log=log,
                                             cfgs={int(c) for c in args.cfgs.split(",")} if args.cfgs else None,
                                             keys=set(args.keys.split(",")) if args.keys else None).items()}
    print(json.dumps({"changes": out, "timings": timings}), flush=True)


if __name__ == "__main__":
    main()
