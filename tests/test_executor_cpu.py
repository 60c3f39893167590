"""Executor on the CPU fake-device backend: single rank and multi-process (gloo) with
cross-device DAG edges, checked against the plain PyTorch reference forward."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_scheduler_amd.models import reference
from distributed_llm_scheduler_amd.parallel import runtime
from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens


def _ref_check(p, ex, store, rid=""):
    tid = f"{rid}output_projection"
    out = ex.output(tid).float()
    B, S = out.shape[0], out.shape[1]
    tok = synthetic_tokens(f"{rid}@tokens", B * S, p.cfg.vocab_size).view(B, S)
    ref = reference.forward(p.cfg, store, tok)
    return (out - ref).abs().max().item(), ref.abs().max().item()


@pytest.mark.parametrize("sched", ["EFT", "MRU_spec", "DFS", "Greedy", "Critical"])
def test_single_rank_matches_reference(sched):
    p = runtime.plan("tiny-gpt2", world=1, scheduler=sched, seq=32, batch=2)
    assert p.completed == p.total
    store = runtime.make_store(p)
    ex = runtime.make_executor(p, 0, "cpu", store)
    ex.step()
    err, scale = _ref_check(p, ex, store)
    assert err < 0.02 * scale


def test_fusion_reduces_kernels():
    fused = runtime.plan("tiny-gpt2", world=1, seq=16)
    plain = runtime.plan("tiny-gpt2", world=1, seq=16, fuse=False)
    n = fused.programs[0].n_kernels
    assert plain.programs[0].n_kernels == fused.total == 19
    # per layer: [ln1+attention+attn_residual], [ln2+ffn_expand+gelu], [ffn_contract+output];
    # the final norm is folded into the LM head: [final_ln+output_projection]
    assert n == 3 * 2 + 2
    kinds = [i.kind for i in fused.programs[0].instrs if i.op == "run"]
    assert kinds[:4] == ["embedding", "layernorm+attention+residual", "layernorm+linear+gelu", "linear+residual"]
    assert kinds[-1] == "layernorm+lm_head"


@pytest.mark.parametrize("sched,cap,residency,mode", [("EFT", 0.00012, "trace", "cold"),
                                                     ("MRU_spec", 0.00012, "auto", "cold"),
                                                     ("EFT", 0.0001, "trace", "warm"),
                                                     ("EFT", 0.00012, "auto", "planned"),
                                                     ("EFT", 0.00008, "auto", "planned")])
def test_capped_plan_steady_state_matches_reference(sched, cap, residency, mode):
    """Under a cap that forces evictions (and, for cyclic EFT, deferred evictions of fused
    norms' weights), repeated steps stay correct and re-fill exactly the planned bytes —
    for a cold-lowered program, a warm-started one (start groups filled once, the program
    restores them at its end) and a planned keep set (kept groups resident, the rest
    streamed)."""
    from distributed_llm_scheduler_amd.parallel.program import steady_fill_bytes

    p = runtime.plan("tiny-gpt2", world=1, scheduler=sched, seq=16, cap_gb=cap, residency=residency)
    assert p.completed == p.total and p.programs[0].counts().get("evict", 0) > 0
    assert p.programs[0].residency == mode
    assert bool(p.programs[0].start_resident) is (mode != "cold")
    store = runtime.make_store(p)
    ex = runtime.make_executor(p, 0, "cpu", store, debug=True)
    for _ in range(3):
        st = ex.step()
    assert st.bytes_filled == steady_fill_bytes(p.programs[0], p.param_bytes)
    err, scale = _ref_check(p, ex, store)
    assert err < 0.02 * scale


def test_memory_cap_enforced_by_scheduler():
    p = runtime.plan("tiny-gpt2", world=1, scheduler="DFS", seq=16, cap_gb=0.00005)
    assert p.completed < p.total
    p2 = runtime.plan("tiny-gpt2", world=1, scheduler="MRU_spec", seq=16, cap_gb=0.00012)
    # MRU evicts and reloads instead of failing; the program replays those evictions
    counts = p2.programs[0].counts()
    assert p2.completed == p2.total and counts.get("evict", 0) > 0
    store = runtime.make_store(p2)
    ex = runtime.make_executor(p2, 0, "cpu", store)
    st = ex.step()
    assert st.param_fills >= counts["load"] - 0  # every planned load is a real fill
    err, scale = _ref_check(p2, ex, store)
    assert err < 0.02 * scale


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, placement, scheduler, q, replicas=2, model="tiny-gpt2", seq=32):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = runtime.plan(model, world=world, scheduler=scheduler, seq=seq, batch=1, replicas=replicas,
                         placement=placement)
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        for _ in range(2):
            st = ex.step()
        res = {"rank": rank, "sends": st.sends, "recvs": st.recvs, "errs": []}
        for rid in (f"r{k}/" for k in range(replicas)):
            if p.placement.get(f"{rid}output_projection") == rank:
                res["errs"].append(_ref_check(p, ex, store, rid))
        q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("placement,scheduler", [("pipeline", "EFT"), ("replica", "EFT"), ("scheduler", "MRU_spec"),
                                                 ("scheduler", "EFT")])
def test_two_ranks_gloo(placement, scheduler):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, placement, scheduler, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    results = [q.get(timeout=5) for _ in range(world)]
    errs = [e for r in results for e in r["errs"]]
    assert len(errs) == 2  # both requests' logits checked on whichever rank owns them
    for err, scale in errs:
        assert err < 0.02 * scale
    if placement == "pipeline":
        assert sum(r["sends"] for r in results) > 0 and sum(r["recvs"] for r in results) > 0


def test_three_ranks_pipeline_reuses_sent_buffers(monkeypatch):
    """GPT-2 on 3 ranks, pipeline placement, 3 micro-batches: rank 1 receives
    r1/layer_3_output into bytes of r0/layer_7_output that are still being sent to rank 2
    (the plan's recv carries a wait for that send); every request's logits must match the
    fp32 reference."""
    monkeypatch.setenv("DLS_PIPELINE_STAGES", "layers")  # the layer-count split makes this buffer reuse
    world, replicas = 3, 3
    p = runtime.plan("gpt2", world=world, seq=64, batch=1, replicas=replicas, placement="pipeline")
    assert any(ins.op == "recv" and ins.wait_sends for pr in p.programs for ins in pr.instrs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, "pipeline", "EFT", q, replicas, "gpt2", 64))
             for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    results = [q.get(timeout=5) for _ in range(world)]
    errs = [e for r in results for e in r["errs"]]
    assert len(errs) == replicas
    for err, scale in errs:
        assert err < 0.02 * scale


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_llama_family_matches_reference(model):
    p = runtime.plan(model, world=1, scheduler="EFT", seq=32, batch=2)
    assert p.completed == p.total
    store = runtime.make_store(p)
    ex = runtime.make_executor(p, 0, "cpu", store)
    ex.step()
    err, scale = _ref_check(p, ex, store)
    assert err < 0.03 * scale


def _ep_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # tiny caps force the scheduler to spread expert nodes over both ranks (EP)
        p = runtime.plan("tiny-mixtral", world=world, scheduler="MRU_spec", seq=32, batch=1, cap_gb=0.0006)
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        st = ex.step()
        experts = {r for t, r in p.placement.items() if "_expert_" in t}
        res = {"rank": rank, "sends": st.sends, "experts_on": sorted(experts), "completed": p.completed,
               "total": p.total, "errs": []}
        if p.placement.get("output_projection") == rank:
            res["errs"].append(_ref_check(p, ex, store))
        q.put(res)
    finally:
        dist.destroy_process_group()


def test_mixtral_expert_parallel_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ep_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs)
    res = [q.get(timeout=5) for _ in range(2)]
    assert res[0]["completed"] == res[0]["total"]
    assert res[0]["experts_on"] == [0, 1]  # experts really are split across GPUs
    assert sum(r["sends"] for r in res) > 0
    errs = [e for r in res for e in r["errs"]]
    assert len(errs) == 1 and errs[0][0] < 0.03 * errs[0][1]


@pytest.mark.parametrize("model", ["tiny-gpt2", "tiny-llama"])
def test_tensor_parallel_transform_single_rank(model):
    p = runtime.plan(model, world=1, seq=32, batch=1, tp=2)
    ids = [t.id for t in p.tasks]
    assert any(i.endswith(".tp1") for i in ids) and any(i.endswith(".sum") for i in ids)
    store = runtime.make_store(p)
    ex = runtime.make_executor(p, 0, "cpu", store)
    ex.step()
    err, scale = _ref_check(p, ex, store)
    assert err < 0.03 * scale


def _tp_worker(rank, world, port, model, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = runtime.plan(model, world=world, seq=32, batch=1, tp=world, placement="tensor")
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        st = ex.step()
        res = {"rank": rank, "sends": st.sends, "recvs": st.recvs, "errs": [],
               "shards": sum(1 for t, r in p.placement.items() if r == rank and ".tp" in t)}
        if p.placement.get("output_projection") == rank:
            res["errs"].append(_ref_check(p, ex, store))
        q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["tiny-gpt2", "tiny-llama"])
def test_tensor_parallel_two_ranks(model):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, model, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs)
    res = sorted([q.get(timeout=5) for _ in range(2)], key=lambda r: r["rank"])
    assert res[1]["shards"] > 0 and res[1]["sends"] > 0 and res[1]["recvs"] > 0
    errs = [e for r in res for e in r["errs"]]
    assert len(errs) == 1 and errs[0][0] < 0.03 * errs[0][1]


def test_plan_checkpoint_resume(tmp_path):
    p = runtime.plan("tiny-gpt2", world=2, scheduler="MRU_spec", seq=16, replicas=2, cap_gb=0.01)
    path = str(tmp_path / "plan.json")
    runtime.save_plan(p, path)
    q = runtime.plan("tiny-gpt2", world=2, scheduler="MRU_spec", seq=16, replicas=2, cap_gb=0.01, resume=path)
    assert q.placement == p.placement and q.order == p.order
    assert [i.__dict__ for i in q.programs[0].instrs] == [i.__dict__ for i in p.programs[0].instrs]
    with pytest.raises(ValueError):
        runtime.plan("tiny-gpt2", world=2, scheduler="MRU_spec", seq=32, replicas=2, cap_gb=0.01, resume=path)
    # a resumed single-rank plan still executes to the reference
    p1 = runtime.plan("tiny-gpt2", world=1, seq=16)
    runtime.save_plan(p1, path)
    q1 = runtime.plan("tiny-gpt2", world=1, seq=16, resume=path)
    store = runtime.make_store(q1)
    ex = runtime.make_executor(q1, 0, "cpu", store)
    ex.step()
    err, scale = _ref_check(q1, ex, store)
    assert err < 0.02 * scale


def test_replan_after_device_loss():
    p = runtime.plan("tiny-gpt2", world=3, seq=16, replicas=3, node_speeds=[1.0, 1.2, 0.8])
    q = runtime.replan(p, [1])
    assert q.world == 2 and q.args["node_speeds"] == [1.0, 0.8]
    assert q.completed == q.total
    assert set(q.placement.values()) <= {0, 1}


def _peer_worker(rank, world, port, model, cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = runtime.plan(model, world=world, seq=16, batch=1, replicas=world, cap_gb=cap, cost_model="bytes")
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        stats = [ex.step() for _ in range(3)]
        res = {"rank": rank, "peer": [s.peer_fills for s in stats], "errs": []}
        for rid in (f"r{k}/" for k in range(world)):
            if p.placement.get(f"{rid}output_projection") == rank:
                res["errs"].append(_ref_check(p, ex, store, rid))
        q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model,cap", [("tiny-gpt2", 0.00012), ("tiny-llama", 0.0002)])
def test_peer_parameter_fills_two_ranks(model, cap):
    """Capped replicas on 2 ranks: steady-state refills of a group the other rank holds are
    received from that rank's arena (RCCL/gloo p2p, the xGMI path) instead of the host image;
    the first step fills from the host (in-place weight transforms happen there). Logits of
    every request must still match the fp32 reference after several steps (for Llama the
    received weights are in their transformed SwiGLU / RoPE form)."""
    from distributed_llm_scheduler_amd.parallel.validate import check_plan

    p = runtime.plan(model, world=2, seq=16, batch=1, replicas=2, cap_gb=cap, cost_model="bytes")
    peers = sum(1 for pr in p.programs for i in pr.instrs if i.op == "load" and i.peer >= 0)
    assert peers > 0 and check_plan(p) == []
    # EFT's planned keep sets differ between the replicas (program.plan_keep_sets shift), so
    # each rank's streamed groups sit resident in the other's arena
    assert all(pr.residency == "planned" for pr in p.programs)
    k0, k1 = (set(pr.start_resident) for pr in p.programs)
    assert {g.split("/", 1)[-1] for g in k0} != {g.split("/", 1)[-1] for g in k1}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer_worker, args=(r, 2, port, model, cap, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    results = [q.get(timeout=5) for _ in range(2)]
    assert sum(r["peer"][0] for r in results) == 0  # first step: host fills only
    assert sum(r["peer"][-1] for r in results) == peers
    errs = [e for r in results for e in r["errs"]]
    assert len(errs) == 2
    for err, scale in errs:
        assert err < 0.02 * scale


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_post_norm_written_by_producer(monkeypatch, model):
    """A norm the next group would run as its own pass is written by the block producing its
    input (residual GEMM / MoE combine) — the norm's own output for a standalone norm group, the
    consumer's scratch for a lead norm. Same outputs as running the norms, and equal to the
    fp32 reference; the first step (weights loaded later) runs the norms itself."""
    from distributed_llm_scheduler_amd.parallel import executor as exm

    outs = {}
    for on in (False, True):
        monkeypatch.setattr(exm, "POST_NORM", "1" if on else "0")
        p = runtime.plan(model, world=1, seq=16)
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, 0, torch.device("cpu"), store)
        assert bool(ex._post_norm) == on
        for _ in range(2):
            ex.step()
        err, scale = _ref_check(p, ex, store)
        assert err < 0.03 * scale, (err, scale)
        outs[on] = ex.output("output_projection").clone()
    assert torch.equal(outs[False], outs[True])


@pytest.mark.parametrize("sched", ["EFT", "MRU_spec"])
def test_post_norm_under_memory_cap(sched):
    """Post-norm pairs with parameter loads / evictions between producer and consumer: the
    producer writes the norm only while the norm's weights are resident, else the consumer runs
    it; repeated capped steps stay equal to the fp32 reference."""
    from distributed_llm_scheduler_amd.models import registry
    from distributed_llm_scheduler_amd.models.params import group_layout

    _, groups, _ = registry.build("tiny-llama", batch=1, seq=16)
    total = sum(group_layout(g)[0] for g in groups.values()) / 1e9
    p = runtime.plan("tiny-llama", world=1, scheduler=sched, seq=16, cap_gb=total * 0.6)
    assert p.completed == p.total and p.programs[0].counts().get("evict", 0) > 0
    store = runtime.make_store(p)
    ex = runtime.make_executor(p, 0, "cpu", store, debug=True)
    assert ex._post_norm
    for _ in range(3):
        ex.step()
    err, scale = _ref_check(p, ex, store)
    assert err < 0.03 * scale, (err, scale)


@pytest.mark.parametrize("model,sched,frac", [("tiny-mixtral", "EFT", 0.35), ("tiny-mixtral", "EFT", 0.6),
                                              ("tiny-mixtral", "MRU_spec", 0.8), ("tiny-llama", "EFT", 0.7),
                                              ("tiny-llama", "MRU_spec", 0.8)])
def test_post_norm_never_reads_stale_weights(model, sched, frac):
    """Cold-lowered capped programs (every step planned from an empty arena, residency
    'trace') load the norm's weight group BETWEEN the producer P and the consumer Q of a
    post-norm pair, and an earlier load can land on the region the group held in the previous
    step. The producer may write the norm only while the group's mapped bytes are really its
    own: every post-norm the producer writes uses weights equal to the store's, for 3 steps,
    and the outputs match the fp32 reference."""
    from distributed_llm_scheduler_amd.models import registry
    from distributed_llm_scheduler_amd.models.params import group_layout
    from distributed_llm_scheduler_amd.parallel.executor import DAGExecutor

    _, groups, _ = registry.build(model, batch=1, seq=16)
    total = sum(group_layout(g)[0] for g in groups.values()) / 1e9
    p = runtime.plan(model, world=1, scheduler=sched, seq=16, cap_gb=total * frac, residency="trace")
    assert p.completed == p.total and p.programs[0].residency == "cold"
    store = runtime.make_store(p)
    ex = runtime.make_executor(p, 0, "cpu", store)
    ins = p.programs[0].instrs
    between = 0
    for i, N in ex._post_norm.items():
        j = next(j for j, q in ex._norm_given.items() if q == N.id)
        between += any(ins[k].op == "load" and ins[k].param in N.params_needed for k in range(i + 1, j))
    assert between > 0, "no post-norm pair with its norm group loaded between producer and consumer"
    written = []
    orig = DAGExecutor._post_norm_out

    def checked(self, out2d):
        r = orig(self, out2d)
        if r is not None:
            W = self._pn.op.weights
            for k in ("w", "b"):
                if k in W:
                    assert torch.equal(self._w(W[k]), store.tensor(W[k]).to(self._w(W[k]).dtype)), \
                        f"post-norm of {self._pn.id} would read stale {k}"
            written.append(self._pn.id)
        return r

    ex._post_norm_out = checked.__get__(ex)
    for _ in range(3):
        ex.step()
    err, scale = _ref_check(p, ex, store)
    assert err < 0.03 * scale, (err, scale)
    for q, (o, n) in ex._region.items():  # no two mapped groups share arena bytes
        for q2, (o2, n2) in ex._region.items():
            assert q == q2 or o + n <= o2 or o2 + n2 <= o, (q, q2)


def _ep_fixed_worker(rank, world, port, q, seq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_scheduler_amd.parallel import executor as exm
        from distributed_llm_scheduler_amd.parallel.validate import check_plan

        exm.RUNNER_CPU = True
        p = runtime.plan("tiny-mixtral", world=world, placement="expert", replicas=1, seq=seq)
        assert not check_plan(p)
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        for _ in range(2):
            st = ex.step()
        widened = 0
        while runtime.ep_widen_on_overflow(ex, dist.group.WORLD):  # capacity edges that overflowed
            widened += 1
            ex.step()
        runner = ex.build_runner()  # an expert-parallel program replays from the native runner
        for _ in range(2):
            st = ex.step()
        assert not runtime.ep_widen_on_overflow(ex, dist.group.WORLD)
        tm = {t.id: t for t in p.tasks}
        wide = ex._ep_full

        def msg_bytes(i):
            grp = (i.task if i.experts else tm[i.task].op.inputs[0], i.peer)
            M = tm[i.task].out_bytes // (2 * tm[i.task].op.out_shape[-1])
            return i.rows * tm[i.task].out_bytes // M if i.rows and grp not in wide else tm[i.task].out_bytes

        edges = [(i.op, i.task, msg_bytes(i)) for i in p.programs[rank].instrs if i.op in ("send", "recv")]
        res = {"rank": rank, "bytes_sent": st.bytes_sent, "bytes_recv": st.bytes_recv, "errs": [],
               "edges": edges, "runner": runner, "issue_mode": ex.issue_mode, "widened": widened,
               "capacity": sum(1 for i in p.programs[rank].instrs if i.rows),
               "experts": sorted(p.placement[t.id] for t in p.tasks if t.op.kind == "moe_expert"),
               "out_bytes": {t.id: t.out_bytes for t in p.tasks}}
        if p.placement.get("output_projection") == rank:
            res["errs"].append(_ref_check(p, ex, store))
        q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_expert_parallel_fixed_size_edges(world):
    """Expert parallelism over 2 / 4 gloo ranks (expert e on rank e % N, the rest of the layer on
    rank 0), replayed by the native step runner: the output matches the fp32 reference, and every
    edge moves a FIXED-size message known when the program is built — the router logits and the
    hidden state's routed rows packed into a capacity buffer (1.25x the expected rows; the whole
    buffer where that is no smaller, or after an overflow widened the group) out to each expert
    rank, each expert's compact output rows back — so no transfer needs routing counts on the
    host (each expert rank routes locally from the logits)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    seq = 24
    procs = [ctx.Process(target=_ep_fixed_worker, args=(r, world, port, q, seq)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    res = sorted([q.get(timeout=5) for _ in range(world)], key=lambda r: r["rank"])
    errs = [e for r in res for e in r["errs"]]
    assert len(errs) == 1 and errs[0][0] < 0.03 * errs[0][1], errs
    assert len(set(res[0]["experts"])) == min(world, 8)
    for r in res:
        assert r["runner"] and r["issue_mode"] == "runner"
        assert r["bytes_sent"] == sum(b for op, _, b in r["edges"] if op == "send")
        assert r["bytes_recv"] == sum(b for op, _, b in r["edges"] if op == "recv")
        assert any("expert" in t for _, t, _ in r["edges"]) or r["rank"] == 0
    if world == 4:  # one expert per rank: the expert edges are capacity messages
        assert all(r["capacity"] > 0 for r in res)


def _runner_worker(rank, world, port, q, model, kw):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_scheduler_amd.parallel import executor as exm
        exm.RUNNER_CPU = True
        p = runtime.plan(model, world=world, seq=16, batch=1, **kw)
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        for _ in range(2):
            py = ex.step()  # the Python issue loop (steady state from the second step)
        assert ex.build_runner()
        for _ in range(3):
            st = ex.step()  # native StepRunner replays
        res = {"rank": rank, "actions": ex._runner.size(), "errs": [],
               "same": (st.sends, st.recvs, st.bytes_sent) == (py.sends, py.recvs, py.bytes_sent)}
        for rid in [f"r{k}/" for k in range(kw.get("replicas", 1))] if kw.get("replicas", 1) > 1 else [""]:
            if p.placement.get(f"{rid}output_projection") == rank:
                res["errs"].append(_ref_check(p, ex, store, rid))
        ex.step(profile=True)  # back to the Python loop after the runner
        q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,kw", [("tiny-llama", dict(replicas=2, placement="pipeline")),
                                      ("tiny-gpt2", dict(tp=2, placement="tensor")),
                                      ("tiny-gpt2", dict(replicas=2, cap_gb=0.00012, cost_model="bytes"))])
def test_native_step_runner_replays_multi_rank_steps(model, kw):
    """The native StepRunner (csrc/kernels/runner.cpp) records one steady-state step of a
    multi-rank program — p2p sends / receives through the c10d ProcessGroup, their waits, and
    (on CPU) the kernel groups as callbacks — and replays it: same transfers, outputs still equal
    to the fp32 reference (pipeline, tensor-parallel and capped replicas with peer parameter
    fills), and the Python loop can resume after it."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_runner_worker, args=(r, world, port, q, model, kw)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    res = [q.get(timeout=5) for _ in range(world)]
    assert all(r["same"] and r["actions"] > 0 for r in res)
    errs = [e for r in res for e in r["errs"]]
    assert errs and all(err < 0.03 * scale for err, scale in errs), errs


@pytest.mark.parametrize("model,kw", [("llama3-8b", dict(placement="pipeline")),
                                      ("mixtral-8x7b", dict(placement="expert", replicas=1)),
                                      ("gpt2", dict(placement="pipeline", replicas=8))])
def test_multi_gpu_placements_keep_the_fused_groups(model, kw):
    """Spreading a DAG over 2 / 8 GPUs (cross-GPU edges = RCCL p2p) keeps every fused kernel
    group of the 1-GPU program: the groups of all ranks add up to the same count (planning only,
    full-size models)."""
    one = sum(runtime.plan(model, world=1, replicas=kw.get("replicas", 1)).stats["kernels_per_rank"])
    for world in (2, 8):
        p = runtime.plan(model, world=world, **kw)
        assert p.stats["cross_gpu_edges"] > 0
        assert sum(p.stats["kernels_per_rank"]) == one, (world, p.stats["kernels_per_rank"], one)


def _ep_dp_worker(rank, world, port, q, seq, max_req=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_llm_scheduler_amd import ops
        from distributed_llm_scheduler_amd.parallel import executor as exm
        from distributed_llm_scheduler_amd.parallel.validate import check_plan

        exm.RUNNER_CPU = True
        if max_req is not None:  # a batch limit below the request count: spans run per node
            ops.XBATCH_MAX_REQ = max_req
        p = runtime.plan("tiny-mixtral", world=world, placement="expert", replicas=world, seq=seq)
        assert not check_plan(p)
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        for _ in range(2):
            ex.step()
        while runtime.ep_widen_on_overflow(ex, dist.group.WORLD):  # capacity edges that overflowed
            ex.step()
        runner = ex.build_runner()
        for _ in range(2):
            ex.step()
        q.put({"rank": rank, "runner": runner, "xbatch": len(ex._xbatch), "layers": p.cfg.n_layer,
               "err": _ref_check(p, ex, store, f"r{rank}/")})
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_expert_dp_gloo_ranks(world):
    """BASELINE config 5 as a process-per-rank job (gloo, 2 / 4 ranks): request r's attention on
    rank r, the experts spread, requests placed layer by layer; every rank runs its experts for
    ALL requests of a layer as one batch (co-run spans), the steps replay from the native runner,
    and every request's logits match the fp32 reference."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ep_dp_worker, args=(r, world, port, q, 24)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    res = sorted([q.get(timeout=5) for _ in range(world)], key=lambda r: r["rank"])
    for r in res:
        assert r["runner"] and r["xbatch"] == r["layers"], r
        err, scale = r["err"]
        assert err < 0.03 * scale, r


@pytest.mark.timeout(300)
def test_expert_dp_gloo_over_batch_limit():
    """More requests per layer than one cross-request batch takes (the index kernel's request
    limit, lowered to 1 here): no span is batched, the members run node by node, and the logits
    still match the fp32 reference."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ep_dp_worker, args=(r, world, port, q, 24, 1)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    res = sorted([q.get(timeout=5) for _ in range(world)], key=lambda r: r["rank"])
    for r in res:
        assert r["runner"] and r["xbatch"] == 0, r
        err, scale = r["err"]
        assert err < 0.03 * scale, r
