"""Per-step device time of the GPT-2 headline step over a long run, from the first replay of its
hipGraph: how many steps the GPU needs to reach its steady state (bench.py's timed window is
whatever the driver asks for — 20 steps after 5 warmup steps in its records).

Each step is bracketed by hipEvents on the executor's stream (the events add nothing to the
graph). Prints the first 60 per-step times, then means over windows."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before the run (GPU idle)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    p = runtime.plan(a.model, world=1, seq=512, batch=1)
    ex = runtime.make_executor(p, 0, dev, runtime.make_store(p, device_init=True), use_graph=True)
    ex.step()
    assert ex.capture()
    torch.cuda.synchronize()
    if a.idle_ms:
        import time
        time.sleep(a.idle_ms / 1e3)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    s = torch.cuda.current_stream(dev)
    ev[0].record(s)
    for i in range(a.steps):
        ex.step()
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
    win = {f"{lo}-{hi}": round(sum(t[lo:hi]) / (hi - lo), 5) for lo, hi in
           [(0, 5), (5, 25), (25, 50), (50, 100), (100, 200), (200, a.steps)] if hi <= a.steps}
    print(json.dumps({"model": a.model, "first": [round(x, 4) for x in t[:60]], "windows_ms": win}))


if __name__ == "__main__":
    main()
