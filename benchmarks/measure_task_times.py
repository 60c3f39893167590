#!/usr/bin/env python3
"""Per-task kernel time of a model's DAG on one MI355X -> ``ops/task_times.json``.

The pipeline-stage partition (runtime.pipeline_stages, csrc/core/partition.h) balances
stages by these times; without the table it falls back to the roofline estimate, which
weighs a GPT-2 layer (45 us measured) at half the LM head (64 us) — the measured table
gets the split right.

Each kernel group of the one-GPU step is timed on its own: the GPU is first put to sleep
for a few hundred microseconds (``torch.cuda._sleep``) so the host has issued the group's
launches before its start event executes, i.e. the bracket holds the group's GPU time and
none of the Python issue loop's host time. A fused group's time is split evenly over its
tasks (a clean pipeline cut never splits a fused group). Median over ``--steps`` steps.

    python benchmarks/measure_task_times.py --models gpt2 gpt2-medium llama3-8b
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402

OUT = os.path.join(ROOT, "distributed_llm_scheduler_amd", "ops", "task_times.json")


def measure(model: str, steps: int, seq: int, sleep_cycles: int) -> dict:
    p = runtime.plan(model, world=1, replicas=1, seq=seq, batch=1)
    store = runtime.make_store(p, device_init=True)
    ex = runtime.make_executor(p, 0, torch.device("cuda:0"), store, use_graph=False)
    for _ in range(3):
        ex.step()
    torch.cuda.synchronize()
    body = ex._issue_run_body

    def slept(i, ins, stats, events):
        if events is not None:
            torch.cuda._sleep(sleep_cycles)  # the group's launches are queued before its start event
        return body(i, ins, stats, events)

    ex._issue_run_body = slept
    groups = {ins.task: ins.group for ins in ex.prog.instrs if ins.op == "run"}
    samples: dict = {}
    for _ in range(steps):
        st = ex.step(profile=True)
        for tid, a, b in st.timeline:
            samples.setdefault(tid, []).append((b - a) * 1e-3)  # ms -> s
    out = {}
    for tid, v in samples.items():
        grp = groups.get(tid, (tid,))
        med = statistics.median(v)
        for t in grp:
            out[t] = med / len(grp)
    for t in p.tasks:  # tasks that ran inside another group's launch (fused away)
        out.setdefault(t.id, 0.0)
    total = sum(out.values())
    print(f"[task_times] {model}: {len(samples)} kernel groups, {total * 1e3:.3f} ms of kernels per step",
          file=sys.stderr, flush=True)
    del ex, store
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["gpt2", "gpt2-medium", "llama3-8b"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--sleep-cycles", type=int, default=2_000_000)
    ap.add_argument("--out", default=OUT)
    args = ap.parse_args()
    try:
        with open(args.out) as f:
            table = json.load(f)
    except (OSError, ValueError):
        table = {}
    keys = []
    for m in args.models:
        key = runtime.task_times_key(runtime.registry.get_config(m).name, args.seq, 1)
        table[key] = {k: round(v, 9) for k, v in measure(m, args.steps, args.seq, args.sleep_cycles).items()}
        keys.append(key)
    table["__meta__"] = {"device": torch.cuda.get_device_name(0), "seq": args.seq, "batch": 1,
                         "date": time.strftime("%Y-%m-%d"), "method": "per kernel group, GPU time (sleep-primed)"}
    with open(args.out, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print(json.dumps({k: round(sum(table[k].values()) * 1e3, 4) for k in keys}))


if __name__ == "__main__":
    main()
