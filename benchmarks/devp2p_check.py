#!/usr/bin/env python3
"""Quick GPU check of the device p2p transport through the single-GPU harness: every case at
2 / 4 ranks, one hipGraph per rank per step; prints errors, host us per step, max rel err."""
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = "16"  # up to 4 rank streams in this process (loopback.py)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

from distributed_llm_scheduler_amd.parallel import devp2p, runtime  # noqa: E402
from distributed_llm_scheduler_amd.parallel.loopback import run_loopback  # noqa: E402
import test_loopback as T  # noqa: E402

devp2p._TICKS = int(float(os.environ.get("TICKS", "2e9")))  # 100 MHz wall-clock ticks per wait
cases = sys.argv[1].split(",") if len(sys.argv) > 1 else T.DEVICE_CASES
worlds = [int(w) for w in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2, 4]
single = os.environ.get("SINGLE", "1") == "1"
nsteps = int(os.environ.get("STEPS", "20"))
# reference: the host cost of issuing a comm-free one-rank step captured as one hipGraph
p1 = runtime.plan("mini-gpt2", world=1, seq=64, batch=2)
ex1 = runtime.make_executor(p1, 0, torch.device("cuda:0"), runtime.make_store(p1), autotune=False)
ex1.step()
ex1.capture()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    ex1.step()
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"one-rank graph (no p2p): host_us={(t1 - t0) / 50 * 1e6:.1f} launches={ex1.launches}", flush=True)
del ex1

for world in worlds:
    for case in cases:
        t0 = time.time()
        p, ids = T._gpu_plan(case, world)
        store = runtime.make_store(p)
        try:
            run = run_loopback(p, "cuda:0", steps=nsteps, warmup=2, store=store, delay_us=50.0, transport="device",
                               single_issue=single)
            errs = [ex.comm.errors() for ex in run.executors]
            errs = f"{errs} warm-up {run.warmup_errors}"
            try:
                w = T._check(p, run, store, ids, 0.03)
                ok = "ok"
            except AssertionError as e:
                w, ok = None, f"MISMATCH {e}"
            print(f"{case} x{world}: {ok} worst={w} errs={errs} modes={run.issue_modes} "
                  f"host_us={[round(h, 1) for h in run.host_us]} launches={[ex.launches for ex in run.executors]} step_ms={[round(m, 3) for m in run.step_ms]} "
                  f"({time.time() - t0:.1f}s)", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{case} x{world}: FAILED {e!r}"[:600], flush=True)
            raise
