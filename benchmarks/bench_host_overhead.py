#!/usr/bin/env python3
"""Host time per executor step, per kernel group, for a program that cannot run as ONE
hipGraph (memory-capped plan whose refills run on the copy stream: DLS_PREFETCH=1), in three
issue modes on the same program:

  eager    the Python issue loop launches every kernel group (no capture)
  segments kernel-group segments replayed as hipGraphs, the Python loop around them (DLS_RUNNER=0)
  runner   the recorded step replayed by the native StepRunner (csrc/kernels/runner.cpp)

    DLS_PREFETCH=1 python benchmarks/bench_host_overhead.py [--model gpt2] [--regime 0.8] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd.models import registry  # noqa: E402
from distributed_llm_scheduler_amd.models.params import group_layout  # noqa: E402
from distributed_llm_scheduler_amd.parallel import executor as exm  # noqa: E402
from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402


def measure(ex, n):
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        ex.step()
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    return sum(host) / n, (time.perf_counter() - t0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--regime", type=float, default=0.8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    tasks, groups, _ = registry.build(a.model, batch=1, seq=512, cost_model="bytes")
    gb = {pid: group_layout(g)[0] / 1e9 for pid, g in groups.items()}
    total = max(t.memory_required + sum(gb[p] for p in t.params_needed) for t in tasks) + sum(gb.values())
    p = runtime.plan(a.model, world=1, scheduler="EFT", cap_gb=total * a.regime, cost_model="bytes")
    dev = torch.device("cuda:0")
    store = runtime.make_store(p, device_init=runtime.device_init_ok(p, 0))
    groups_n = p.programs[0].n_kernels
    out = {"model": a.model, "regime": a.regime, "kernel_groups": groups_n,
           "instructions": len(p.programs[0].instrs), "prefetch": os.environ.get("DLS_PREFETCH", "auto")}
    for mode in ("eager", "segments", "runner"):
        exm.RUNNER = mode == "runner"
        exm.RUNNER_MODE = "1" if mode == "runner" else "0"  # no measured fallback here
        ex = runtime.make_executor(p, 0, dev, store, use_graph=mode != "eager")
        for _ in range(3):
            ex.step()
        if mode != "eager":
            ex.capture()
            ex.step()
        assert (ex._runner is not None) == (mode == "runner"), mode
        host, wall = measure(ex, a.steps)
        out[mode] = {"host_ms_per_step": round(host * 1e3, 3), "wall_ms_per_step": round(wall * 1e3, 3),
                     "host_us_per_group": round(host * 1e6 / groups_n, 2),
                     "segments": len(ex._segments)}
        print(f"{a.model} regime {a.regime} {mode:9s}: host {host * 1e3:.3f} ms/step = "
              f"{host * 1e6 / groups_n:.1f} us per kernel group ({groups_n} groups), wall {wall * 1e3:.3f} ms/step",
              flush=True)
        del ex
        torch.cuda.synchronize()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
