#!/usr/bin/env python3
"""Host -> HBM parameter-refill bandwidth: hipMemcpyAsync (tensor.copy_ from pinned memory)
vs the host-pull kernel (ops.host_pull) at several grid sizes, for the group sizes the capped
plans re-fill (GPT-2: 6 KB norms ... 77 MB embedding). hipEvent-timed, 20 reps each; also in
a captured hipGraph (the executor's steady state)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd import ops  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def graphed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return timed(g.replay, reps)


def main():
    ext = ops.ext()
    out = []
    for mb in (0.25, 2.4, 9.4, 37.8, 77.2):
        n = int(mb * 1e6) // 256 * 256
        src = torch.randint(0, 255, (n,), dtype=torch.uint8).pin_memory()
        dst = torch.empty(n, dtype=torch.uint8, device="cuda")
        row = {"MB": mb}
        ms = timed(lambda: dst.copy_(src, non_blocking=True))
        row["memcpy_GBps"] = round(n / ms / 1e6, 1)
        row["memcpy_graph_GBps"] = round(n / graphed(lambda: dst.copy_(src, non_blocking=True)) / 1e6, 1)
        for blocks in (32, 64, 128, 256, 512, 1024):
            ms = timed(lambda: ext.host_pull(dst, src, blocks))
            row[f"pull{blocks}_GBps"] = round(n / ms / 1e6, 1)
        best = max((k for k in row if k.startswith("pull")), key=lambda k: row[k])
        nb = int(best[4:].split("_")[0])
        row["pull_best_graph_GBps"] = round(n / graphed(lambda: ext.host_pull(dst, src, nb)) / 1e6, 1)
        assert torch.equal(dst.cpu(), src), "host_pull copied wrong bytes"
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
