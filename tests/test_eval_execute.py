"""Executed evaluation (eval/execute.py, ``simulation.py --execute``): each policy's
placement of a model DAG under the reference's memory regimes is RUN by the executor,
and the raw_results.csv row carries the measured makespan."""
import os
import socket

import pandas as pd
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_scheduler_amd.eval import execute
from distributed_llm_scheduler_amd.eval.simulation import EXTRA_COLUMNS, REF_COLUMNS


def test_single_device_regimes(tmp_path):
    rows = execute.main("tiny-gpt2", ["DFS", "MRU_spec"], (1.0, 0.8), steps=1, warmup=1, seq=16,
                        out_dir=str(tmp_path), plot=False)
    got = {(r.scheduler_name, r.memory_regime): r for r in rows}
    # the reference's completion semantics, now executed: at 80 % DFS fails tasks, MRU
    # completes everything by evicting and re-loading parameters (real refills per step)
    assert got[("DFS", 0.8)].completed_tasks < got[("DFS", 0.8)].total_tasks
    mru = got[("MRU_spec", 0.8)]
    assert mru.completed_tasks == mru.total_tasks and mru.param_evictions > 0 and mru.param_fill_bytes > 0
    for r in rows:
        assert r.wall_makespan_ms > 0 and r.hbm_peak_gb > 0 and r.device == "cpu" and r.dag_type == "LLM-tiny-gpt2"
    df = pd.read_csv(tmp_path / "raw_results.csv")
    assert list(df.columns) == REF_COLUMNS + EXTRA_COLUMNS
    assert len(df) == 4 and df["wall_makespan_ms"].notna().all()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = execute.main("tiny-gpt2", ["MRU_spec", "Critical"], (0.8,), steps=1, warmup=1, seq=16, out_dir=out,
                            plot=False)
        q.put((rank, [(r.scheduler_name, r.completed_tasks, r.total_tasks, r.wall_makespan_ms, r.num_nodes,
                       r.bytes_moved_p2p) for r in rows]))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res[0] == res[1]  # max/sum-reduced metrics: every rank reports the same row
    for name, done, total, wall, n, p2p in res[0]:
        assert n == 2 and wall > 0
    mru = [r for r in res[0] if r[0] == "MRU_spec"][0]
    assert mru[1] == mru[2]
    df = pd.read_csv(tmp_path / "raw_results.csv")
    assert (df["num_nodes"] == 2).all()
