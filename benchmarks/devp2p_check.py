#!/usr/bin/env python3
"""Quick GPU check of the device p2p transport through the single-GPU harness: every case at
2 / 4 ranks, one hipGraph per rank per step; prints errors, host us per step, max rel err."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")  # up to 4 rank streams in this process (loopback.py)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import torch  # noqa: E402

from distributed_llm_scheduler_amd.parallel import devp2p, runtime  # noqa: E402
from distributed_llm_scheduler_amd.parallel.loopback import run_loopback  # noqa: E402
import test_loopback as T  # noqa: E402

devp2p._TICKS = int(2e8)
cases = sys.argv[1].split(",") if len(sys.argv) > 1 else T.DEVICE_CASES
worlds = [int(w) for w in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2, 4]
for world in worlds:
    for case in cases:
        t0 = time.time()
        p, ids = T._gpu_plan(case, world)
        store = runtime.make_store(p)
        try:
            run = run_loopback(p, "cuda:0", steps=20, warmup=2, store=store, delay_us=50.0, transport="device",
                               single_issue=True)
            errs = [ex.comm.errors() for ex in run.executors]
            try:
                w = T._check(p, run, store, ids, 0.03)
                ok = "ok"
            except AssertionError as e:
                w, ok = None, f"MISMATCH {e}"
            print(f"{case} x{world}: {ok} worst={w} errs={errs} modes={run.issue_modes} "
                  f"host_us={[round(h, 1) for h in run.host_us]} step_ms={[round(m, 3) for m in run.step_ms]} "
                  f"({time.time() - t0:.1f}s)", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{case} x{world}: FAILED {e!r}"[:600], flush=True)
            raise
