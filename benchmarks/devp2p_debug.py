#!/usr/bin/env python3
"""Edge-by-edge check of the device p2p transport (eager steps): the producer snapshots each
sent region right before its notify, the consumer snapshots its region right after the pull;
any slot whose two snapshots differ is printed (case, world from argv)."""
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from distributed_llm_scheduler_amd.parallel import devp2p, runtime  # noqa: E402
from distributed_llm_scheduler_amd.parallel.loopback import run_loopback  # noqa: E402
import test_loopback as T  # noqa: E402

devp2p._TICKS = int(2e9)
case, world = sys.argv[1], int(sys.argv[2])
delay = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
capture = len(sys.argv) > 4 and sys.argv[4] == "graph"
sent, got = {}, {}
step_of = {}
orig_isend, orig_irecv = devp2p.DeviceComm.isend, devp2p.DeviceComm.irecv
orig_wait = devp2p._RecvWork.wait


def isend(self, buf, peer, key=None):
    k = (self.rank, peer, key)
    n = step_of[self.rank]
    arena, off, nb = self.w.sources[k]
    src = torch.empty(nb, dtype=torch.uint8, device=buf.device)
    base = self.w.bases[self.rank][arena]
    reg = (self.w._exported[self.rank][arena])[off:off + nb]
    src.copy_(reg)
    sent[(k, n)] = src
    return orig_isend(self, buf, peer, key)


def irecv(self, buf, peer, key=None):
    w = orig_irecv(self, buf, peer, key)
    w.__dict__ if hasattr(w, "__dict__") else None
    return _W(w, (peer, self.rank, key), step_of[self.rank], buf)


class _W:
    def __init__(self, w, k, n, buf):
        self.w, self.k, self.n, self.buf = w, k, n, buf

    def wait(self):
        self.w.wait()
        got[(self.k, self.n)] = self.buf.clone()


def begin(self):
    step_of[self.rank] = step_of.get(self.rank, 0) + 1
    self.e.p2p_tick(self.mb.step)


devp2p.DeviceComm.isend, devp2p.DeviceComm.irecv, devp2p.DeviceComm.begin_step = isend, irecv, begin
p, ids = T._gpu_plan(case, world)
store = runtime.make_store(p)
run = run_loopback(p, "cuda:0", steps=2, warmup=1, capture=capture, store=store, delay_us=delay, transport="device")
torch.cuda.synchronize()
bad = 0
for (k, n), dst in sorted(got.items(), key=lambda kv: (kv[0][1], str(kv[0][0]))):
    src = sent.get((k, n))
    if src is None:
        print("no snapshot for", k, n)
        continue
    if not torch.equal(src, dst):
        bad += 1
        diff = (src != dst).nonzero()
        ff = float((dst == 0xFF).float().mean())
        same = [f"{kk[2]}@{nn}" for (kk, nn), v in sent.items() if v.numel() == dst.numel() and torch.equal(v, dst)]
        later = sent.get((k, n + 1))
        print(f"BAD step {n} {k}: {diff.numel()} bytes differ, first at {int(diff[0])} of {src.numel()}; "
              f"dst 0xFF frac {ff:.3f}; dst equals snapshots {same[:4]}; "
              f"src(step {n}) == src(step {n + 1}): {None if later is None else torch.equal(later, src)}")
print(f"{case} x{world}: {len(got)} pulls checked, {bad} bad; errors {[ex.comm.errors() for ex in run.executors]}")
try:
    print("worst", T._check(p, run, store, ids, 0.03))
except AssertionError as e:
    print("MISMATCH", e)
