#!/usr/bin/env python3
"""Dump every rank's device-p2p mailbox (step counter, ready / ack flags) after each eager step
of a loopback run (case, world from argv): flags must equal the step number everywhere."""
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from distributed_llm_scheduler_amd.parallel import devp2p, runtime  # noqa: E402
from distributed_llm_scheduler_amd.parallel import loopback as lb  # noqa: E402
import test_loopback as T  # noqa: E402

devp2p._TICKS = int(2e9)
case, world = sys.argv[1], int(sys.argv[2])
p, ids = T._gpu_plan(case, world)
store = runtime.make_store(p)
worlds = []
orig = devp2p.DeviceP2PWorld.__init__


def init(self, *a, **k):
    orig(self, *a, **k)
    worlds.append(self)


devp2p.DeviceP2PWorld.__init__ = init
for steps in (1, 2):
    run = lb.run_loopback(p, "cuda:0", steps=steps, warmup=0, capture=False, store=store, delay_us=50.0,
                          transport="device")
    torch.cuda.synchronize()
    w = worlds[-1]
    inv = {v: k for k, v in w.slots.items()}
    for r in range(world):
        m = w.mail[r]
        print(f"[{steps} steps] rank {r}: step={int(m.step.item())} err={int(m.err.item())} "
              f"ready={m.ready.tolist()} ack={m.ack.tolist()}")
    print("slots:", [(s, inv[s][0], inv[s][1], inv[s][2][1]) for s in range(len(inv))][:12])
    try:
        print("worst", T._check(p, run, store, ids, 0.03))
    except AssertionError as e:
        print("MISMATCH", e)
