#!/usr/bin/env python3
"""Host (Python) time per eager executor step vs GPU time per step, for a capped Llama-3-8B
plan (planned residency + copy-stream prefetch => eager): is the eager step host-bound?
    python benchmarks/bench_host_overhead.py [regime]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd.models import registry  # noqa: E402
from distributed_llm_scheduler_amd.models.params import group_layout  # noqa: E402
from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402


def main():
    regime = float(sys.argv[1]) if len(sys.argv) > 1 else 0.9
    model = sys.argv[2] if len(sys.argv) > 2 else "llama3-8b"
    tasks, groups, _ = registry.build(model, batch=1, seq=512, cost_model="bytes")
    gb = {pid: group_layout(g)[0] / 1e9 for pid, g in groups.items()}
    total = max(t.memory_required + sum(gb[p] for p in t.params_needed) for t in tasks) + sum(gb.values())
    p = runtime.plan(model, world=1, scheduler="EFT", cap_gb=total * regime, cost_model="bytes")
    dev = torch.device("cuda:0")
    store = runtime.make_store(p, device_init=runtime.device_init_ok(p, 0))
    ex = runtime.make_executor(p, 0, dev, store)
    for _ in range(3):
        ex.step()
    torch.cuda.synchronize()
    if os.environ.get("DLS_CAPTURE") == "1":  # hipGraph (segments) as bench.py does
        print("captured:", ex.capture(), "segments:", len(ex._segments), flush=True)
        ex.step()
        torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    host = []
    for _ in range(n):
        a = time.perf_counter()
        ex.step()
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    print(f"{model} regime {regime}: prefetch={ex._copy_stream is not None} host {sum(host) / n * 1e3:.2f} ms/step "
          f"(min {min(host) * 1e3:.2f}), wall {wall * 1e3:.2f} ms/step, kernels/step {p.programs[0].n_kernels}",
          flush=True)
    if os.environ.get("DLS_HOST_PROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(n):
            ex.step()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
