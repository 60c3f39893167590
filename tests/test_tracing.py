"""Measured timelines, Chrome-trace export and roctx plumbing (CPU backend)."""
import json
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_scheduler_amd.parallel import runtime
from distributed_llm_scheduler_amd.utils import tracing
from test_executor_cpu import _free_port


def test_profile_events_single_rank(tmp_path):
    p = runtime.plan("tiny-gpt2", world=1, seq=16)
    ex = runtime.make_executor(p, 0, "cpu", trace=True)
    st = ex.step(profile=True)
    kinds = {c for _, c, _, _ in st.events}
    assert {"kernel", "load"} <= kinds
    assert len(st.timeline) == p.programs[0].n_kernels
    assert all(b >= a >= 0 for _, a, b in st.timeline)
    starts = [a for _, a, _ in st.timeline]
    assert starts == sorted(starts)
    st2 = ex.step(profile=True)  # steady state: parameters resident, no fills
    assert not [e for e in st2.events if e[1] == "load"]
    doc = tracing.chrome_trace({0: st.events}, str(tmp_path / "t.json"), meta={"model": "tiny-gpt2"})
    on_disk = json.load(open(tmp_path / "t.json"))
    assert on_disk == doc
    xs = [e for e in doc["traceEvents"] if e["ph"] == "X"]
    assert len(xs) == len(st.events) and all(e["dur"] >= 0 for e in xs)
    summ = tracing.summarize(st.events)
    assert summ["span"] >= summ["kernel"] * 0.0 and summ["kernel"] > 0


def test_roctx_ranges_are_balanced():
    tracing.Roctx.push("x")
    tracing.Roctx.mark("m")
    tracing.Roctx.pop()
    with tracing.roctx_range("y"):
        pass
    assert isinstance(tracing.Roctx.available(), bool)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = runtime.plan("tiny-gpt2", world=world, seq=16, placement="pipeline")
        ex = runtime.make_executor(p, rank, "cpu", pg=dist.group.WORLD)
        st = ex.step(profile=True)
        evs = [None] * world
        dist.all_gather_object(evs, st.events)
        if rank == 0:
            q.put(evs)
    finally:
        dist.destroy_process_group()


def test_two_rank_trace_has_p2p_rows():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs)
    evs = q.get(timeout=5)
    cats = [{c for _, c, _, _ in e} for e in evs]
    assert "send" in cats[0] and "recv" in cats[1]
    doc = tracing.chrome_trace(dict(enumerate(evs)))
    assert {e["pid"] for e in doc["traceEvents"] if e["ph"] == "X"} == {0, 1}
