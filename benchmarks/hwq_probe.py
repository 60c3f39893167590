#!/usr/bin/env python3
"""Which torch streams of ONE process share a hardware queue? A one-wave kernel on stream 0
spins on a flag that a kernel on stream k sets; if the two streams share a queue, the setter
waits behind the spinner until the spin's timeout (0.5 s here). Prints, per k, the time the
pair took. (The single-GPU multi-rank harness with the device p2p transport needs every rank's
stream on a queue of its own: parallel/loopback.py.)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if len(sys.argv) > 1:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[1]

import torch  # noqa: E402

from distributed_llm_scheduler_amd import ops  # noqa: E402

e = ops.ext()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
mode = sys.argv[3] if len(sys.argv) > 3 else "pool"
dev = torch.device("cuda:0")
if mode == "pool":
    streams = [torch.cuda.Stream(dev) for _ in range(n)]
else:  # raw hipStreamCreate'd streams, not torch's pool
    streams = [torch.cuda.ExternalStream(e.stream_create()) for _ in range(n)] if hasattr(e, "stream_create") else []
flag = torch.zeros(1, dtype=torch.int64, device=dev)
step = torch.ones(1, dtype=torch.int64, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
res = []
for k in range(1, len(streams)):
    flag.zero_()
    err.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(streams[0]):
        e.p2p_wait(flag, step, err, int(0.5e8), 4)  # 0.5 s timeout
    with torch.cuda.stream(streams[k]):
        e.p2p_notify(flag.data_ptr(), step)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e3
    res.append((k, round(dt, 2), int(err.item())))
print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')} streams={len(streams)} mode={mode}: "
      + " ".join(f"{k}:{dt}ms{'(TIMEOUT)' if er else ''}" for k, dt, er in res), flush=True)
