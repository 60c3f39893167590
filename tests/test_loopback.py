"""The multi-GPU executor path on ONE device: a world-rank job in one process, every rank its
own executor / stream / host thread, DAG edges through the loopback hub with RCCL's p2p
semantics (parallel/loopback.py). On the GPU every transfer runs behind a spinning delay kernel
and every receive buffer is poisoned with NaN when posted, so a consumer that is not ordered
after its transfer (or a producer that overwrites a buffer before its send completed) breaks the
fp32 comparison — device-side asynchrony a gloo job cannot show. The segment hipGraphs and the
native step runner's SEND / RECV / WORK_WAIT / group actions run exactly as in an RCCL job.

Reference parity: the reference's experiments are all multi-node (/root/reference/
simulation.py:376 node_configs [2, 4, 8]; test_gpt2.py:277-283, four laptops)."""
import pytest
import torch

from distributed_llm_scheduler_amd.eval.execute import regime_node_spec
from distributed_llm_scheduler_amd.models import reference
from distributed_llm_scheduler_amd.parallel import runtime
from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens
from distributed_llm_scheduler_amd.parallel.loopback import run_loopback

# (model, plan kwargs, output task ids): every placement whose programs carry p2p edges
CASES = {
    "pipeline": ("tiny-gpt2", dict(placement="pipeline", replicas=2), ["r0/output_projection", "r1/output_projection"]),
    # the same micro-batches merged into ONE batch-2 request before placement (plan merge_mb)
    "pipeline_merged": ("tiny-gpt2", dict(placement="pipeline", replicas=2, merge_mb=2),
                        ["r0/output_projection", "r1/output_projection"]),
    "tensor": ("tiny-llama", dict(placement="tensor", tp=2), ["output_projection"]),
    "sequence": ("tiny-gpt2", dict(placement="sequence", sp=2), None),
    "expert": ("tiny-mixtral", dict(placement="expert", replicas=1), ["output_projection"]),
    # config 5: data-parallel attention (one request per GPU) + expert parallelism; every GPU runs
    # its experts for all requests of a layer as ONE grouped launch pair (program.plan_coruns)
    "expert_dp": ("tiny-mixtral", dict(placement="expert", replicas="world"), "replicas"),
    # the reference's experiment: ONE DAG over the nodes under its 80 % regime (bench.py capped)
    "capped_one_dag": ("tiny-gpt2", dict(scheduler="MRU_spec", regime=0.8), ["output_projection"]),
    # the same experiment placed by EFT's steady-state partition (a pipeline of capped stages)
    "capped_eft": ("tiny-gpt2", dict(scheduler="EFT", regime=0.8), ["output_projection"]),
    # capped replicas: steady-state refills of a group a peer holds come from the peer's HBM
    # (program.plan_peer_fills, the xGMI path); the cap is a fraction of the model's parameters
    "peer_fill": ("tiny-gpt2", dict(replicas="world", cap_frac=0.7, cost_model="bytes"), "replicas"),
}


def _plan(case, world, seq, batch=1, gpu=False):
    model, kw, ids = CASES[case]
    if gpu:  # the smallest shapes the GPU kernels take (head_dim 64)
        model = model.replace("tiny-", "mini-")
    kw = dict(kw)
    if case == "sequence" and world == 4:
        kw["sp"] = 4
    if "regime" in kw:
        spec = regime_node_spec(model, kw.pop("regime"), world, batch=batch, seq=seq)
        kw.update(cap_gb=[m for m, _ in spec], node_speeds=[v for _, v in spec], cost_model="reference")
    if kw.get("replicas") == "world":
        kw["replicas"] = world
    if "cap_frac" in kw:
        total = sum(runtime.plan(model, world=1, seq=seq, batch=batch).param_bytes.values())
        kw["cap_gb"] = kw.pop("cap_frac") * total / 1e9
    if ids == "replicas":
        ids = [f"r{k}/output_projection" for k in range(world)]
    return runtime.plan(model, world=world, seq=seq, batch=batch, **kw), ids


def _p2p_work(p):
    """Cross-rank traffic the plan carries: DAG edges plus parameter groups filled from a peer."""
    peer = sum(1 for pr in p.programs for i in pr.instrs if i.op == "load" and i.peer >= 0)
    return p.stats["cross_gpu_edges"] + peer


def _logits(p, run, ids):
    """{request prefix: [B, S, V] logits}, gathered from whichever rank produced them."""
    def out(tid):
        return run.executors[p.owner(tid)].output(tid).float().cpu()
    if ids is None:  # sequence chunks: the request's logits are the chunks' rows in order
        P = sum(1 for t in p.tasks if t.id.startswith("output_projection.sp"))
        return {"": torch.cat([out(f"output_projection.sp{c}") for c in range(P)], dim=1)}
    return {(t.split("/")[0] + "/" if "/" in t else ""): out(t) for t in ids}


def _check(p, run, store, ids, tol):
    """Max relative error of every request's logits vs the fp32 reference forward."""
    worst = 0.0
    for rid, out in _logits(p, run, ids).items():
        assert torch.isfinite(out).all(), f"{rid}: non-finite logits (a consumer read a poisoned receive buffer)"
        B, S = out.shape[0], out.shape[1]
        tok = synthetic_tokens(f"{rid}@tokens", B * S, p.cfg.vocab_size).view(B, S)
        margins = []
        ref = reference.forward(p.cfg, store, tok, router_margins=margins)
        scale = ref.abs().max().item()
        row = (out - ref).abs().amax(-1) / scale
        if margins:  # MoE: only rows whose k-th / (k+1)-th router logits nearly tie may route
            risky = torch.stack([m.abs() < 0.05 for m in margins]).any(0)  # differently in bf16
            assert (row[risky] > tol).float().mean().item() < 0.5 if risky.any() else True
            row = row[~risky]
        worst = max(worst, row.max().item())
    assert worst < tol, worst
    return worst


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("cpu_runner", [False, True])
def test_loopback_cpu(case, world, cpu_runner):
    p, ids = _plan(case, world, 32 if case == "sequence" else 16)
    assert _p2p_work(p) > 0 and p.completed == p.total
    store = runtime.make_store(p)
    run = run_loopback(p, "cpu", steps=2, warmup=2, store=store, cpu_runner=cpu_runner)
    assert run.hub.transfers > 0 and run.hub.outstanding() == 0
    if case == "peer_fill":
        assert sum(s.peer_fills for s in run.stats) > 0, "no parameter group came from a peer"
    if cpu_runner:
        assert all(m == "runner" for m in run.issue_modes)
    _check(p, run, store, ids, 0.03)


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("world", [2, 4])
def test_loopback_cpu_device_transport(case, world):
    """The device transport's protocol with host waits (devp2p.HostP2PWorld): every placement
    runs the executor's device-transport paths on the CPU — regions pulled at their post, routed
    expert rows pulled once their routing is here, sends completed by the consumer's pull — with
    NaN-poisoned receive regions, no wait timing out, and logits matching fp32."""
    p, ids = _plan(case, world, 32 if case == "sequence" else 16)
    store = runtime.make_store(p)
    run = run_loopback(p, "cpu", steps=2, warmup=1, store=store, transport="device", timeout_s=20.0)
    assert [ex.comm.errors() for ex in run.executors] == [0] * world
    assert run.warmup_errors == [0] * world
    assert sum(ex.comm.bytes_pulled() for ex in run.executors) > 0 or case == "peer_fill"
    _check(p, run, store, ids, 0.03)


def test_loopback_cpu_device_transport_catches_late_expert_pulls(monkeypatch):
    """Negative control of the host device transport: with expert outputs pulled at the combine
    again (the rule before round 5), the layer-major config-5 plan stalls — both ranks wait for
    the ack of a region the other pulls only later — and the waits time out into the error words
    (validate.device_deadlock_check(eager=False) predicts it)."""
    from distributed_llm_scheduler_amd.parallel import executor as exm
    p, ids = _plan("expert_dp", 2, 16)
    store = runtime.make_store(p)
    orig = exm.DAGExecutor._pull_expert_rows

    def late(self, x, w):  # defer to the combine, as the old executor did
        self._deferred[x] = w

    def combine(self, t, out, _orig=exm.DAGExecutor._moe_combine):
        a = t.op.attrs
        off = self._moe_route(t.op.inputs[-2], a["n_experts"], a["top_k"])[4]
        for x in t.op.inputs[:-2]:
            w = self._deferred.pop(x, None)
            if w is not None:
                v = self._views[x]
                w.pull_rows(self._act_region(x), v.shape[-1] * v.element_size(), None, off, self._exp_ids[x],
                            v.numel() // v.shape[-1])
        _orig(self, t, out)

    monkeypatch.setattr(exm.DAGExecutor, "_pull_expert_rows", late)
    monkeypatch.setattr(exm.DAGExecutor, "_moe_combine", combine)
    # the stalled wait fails the step loudly (executor.TransportError, re-raised by the harness)
    with pytest.raises(RuntimeError, match="timed out") as ei:
        run_loopback(p, "cpu", steps=1, warmup=0, store=store, transport="device", timeout_s=2.0)
    assert isinstance(ei.value.__cause__, exm.TransportError), repr(ei.value.__cause__)
    assert orig is not late


@pytest.mark.parametrize("world", [2, 4])
def test_expert_dp_batches_every_request_per_layer(world, monkeypatch):
    """Config 5 (data-parallel attention + expert parallelism): the requests are placed layer by
    layer, so every rank's program holds one co-run span per MoE layer with ALL requests'
    nodes of its experts, the executor issues each span as one grouped batch, and per-node
    launches (DLS_MOE_XBATCH=0) give the same logits."""
    from distributed_llm_scheduler_amd.parallel import executor as exm
    p, ids = _plan("expert_dp", world, 16)
    L, E = p.cfg.n_layer, p.cfg.n_experts
    for pr in p.programs:
        assert len(pr.coruns) == L, (pr.rank, pr.coruns)
        assert all(len(span) == world * (E // world) for span in pr.coruns)
        assert all({t.split("/")[0] for t in span} == {f"r{k}" for k in range(world)} for span in pr.coruns)
    store = runtime.make_store(p)
    outs = {}
    for on in (True, False):
        monkeypatch.setattr(exm, "MOE_XBATCH", on)
        run = run_loopback(p, "cpu", steps=1, warmup=1, store=store)
        assert all(len(ex._xbatch) == (L if on else 0) for ex in run.executors)
        outs[on] = _logits(p, run, ids)
        _check(p, run, store, ids, 0.03)
    for rid in outs[True]:
        assert torch.allclose(outs[True][rid], outs[False][rid], atol=2e-2, rtol=0), rid


# --------------------------------------------------------------------------- GPU
def gpu(f):
    """GPU harness tests: several ranks capture on threads of ONE process, so each runs in a
    fresh child process of its own with GPU_MAX_HW_QUEUES=16 (tests/conftest.py ``isolated``)."""
    return pytest.mark.isolated(pytest.mark.gpu(f))


def _gpu_plan(case, world, seq=64):
    return _plan(case, world, seq, batch=2, gpu=True)


@gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("world", [2, 4])
def test_loopback_gpu(case, world):
    """Every p2p placement at 2 / 4 ranks on one MI355X: segment hipGraphs + the native step
    runner on every rank, 50 us of delay in front of every transfer, poisoned receive buffers —
    the logits match fp32."""
    p, ids = _gpu_plan(case, world)
    assert _p2p_work(p) > 0
    store = runtime.make_store(p)
    run = run_loopback(p, "cuda:0", steps=3, warmup=2, store=store, delay_us=50.0)
    assert run.hub.transfers > 0 and run.hub.outstanding() == 0
    comm_ranks = [r for r in range(world) if p.programs[r].has_comm]
    assert comm_ranks and all(run.issue_modes[r] == "runner" for r in comm_ranks), run.issue_modes
    if case == "peer_fill":
        assert sum(s.peer_fills for s in run.stats) > 0, "no parameter group came from a peer"
    _check(p, run, store, ids, 0.03)


@gpu
@pytest.mark.timeout(240)
def test_loopback_gpu_catches_missing_wait():
    """Negative control: with the consumer's receive wait removed on one rank, the same run reads
    the poisoned buffer (or a half-landed transfer) and the check fails — the harness has teeth."""
    p, ids = _gpu_plan("pipeline", 2)
    store = runtime.make_store(p)

    def drop_waits(exs):
        ex = exs[1]
        orig = ex._pre_run

        def pre_run(ins, recv_work, events):  # receives posted, never waited for before their consumer
            saved = dict(recv_work)
            recv_work.clear()
            orig(ins, recv_work, events)
            recv_work.update(saved)
        ex._pre_run = pre_run

    run = run_loopback(p, "cuda:0", steps=1, warmup=1, capture=False, store=store, delay_us=200.0,
                       before_steps=drop_waits)
    with pytest.raises(AssertionError):
        _check(p, run, store, ids, 0.03)


@gpu
@pytest.mark.timeout(240)
def test_loopback_gpu_expert_parallel_no_host_sync():
    """Expert parallelism replays with no device->host synchronisation inside a step: every edge
    is a fixed-size buffer, each expert rank routes from the received logits on the device
    (torch's sync debug mode raises on any synchronising call during the steps)."""
    p, ids = _gpu_plan("expert", 4)
    store = runtime.make_store(p)
    run = run_loopback(p, "cuda:0", steps=3, warmup=2, capture=False, store=store, sync_debug=True)
    assert all(s is not None for s in run.stats)
    _check(p, run, store, ids, 0.03)


@gpu
@pytest.mark.timeout(240)
def test_loopback_gpu_mixed_issue_modes():
    """ranks that disagree on the native runner stay in p2p step. Rank 1 cannot record
    a runner (forced), rank 0 can: build_runner executes the recorded step on rank 0, and rank 1
    runs one Python-loop step in its place, so their transfers still pair step by step."""
    p, ids = _gpu_plan("pipeline", 2)
    store = runtime.make_store(p)

    def refuse_on_rank1(exs):
        exs[1]._runner_ok = lambda: False

    run = run_loopback(p, "cuda:0", steps=3, warmup=2, store=store, delay_us=50.0, before_steps=refuse_on_rank1)
    assert run.issue_modes[0] == "runner" and run.issue_modes[1] != "runner", run.issue_modes
    assert run.hub.outstanding() == 0
    _check(p, run, store, ids, 0.03)


# ------------------------------------------------------------------ device transport (GPU)
# every placement's edges moved by kernels (parallel/devp2p.py): notify / pull / ack flags with
# no host pairing, each rank's WHOLE step captured into one hipGraph
DEVICE_CASES = ["pipeline", "pipeline_merged", "capped_eft", "capped_one_dag", "tensor", "sequence", "expert",
                "expert_dp", "peer_fill"]


@gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("case", DEVICE_CASES)
@pytest.mark.parametrize("world", [2, 4])
def test_loopback_gpu_device_transport(case, world, monkeypatch):
    """Each rank replays ONE hipGraph per step — kernels, notifies, pulls and acks — with 50 us
    of delay in front of every notify and NaN-poisoned receive regions; no wait timed out, the
    logits match fp32, and issuing a step costs the host one graph launch whatever the edge
    count (measured 13-42 us per step for 57-75 kernel nodes; round-4 runner: 10-16 us per
    SEGMENT)."""
    from distributed_llm_scheduler_amd.parallel import devp2p
    # 20 s: a rank's first (cold) step loads code objects while its peers already wait
    monkeypatch.setattr(devp2p, "_TICKS", int(2e9))
    p, ids = _gpu_plan(case, world)
    assert _p2p_work(p) > 0
    store = runtime.make_store(p)
    run = run_loopback(p, "cuda:0", steps=20, warmup=2, store=store, delay_us=50.0, transport="device",
                       single_issue=True)
    assert run.issue_modes == ["graph"] * world, run.issue_modes
    assert run.warmup_errors == [0] * world and [ex.comm.errors() for ex in run.executors] == [0] * world
    # ROCm's hipGraphLaunch itself costs ~0.3 us per kernel node: the config-5 plans (every rank
    # a request's whole layer chain plus its experts for all requests) carry 75-139 nodes
    nodes = max(ex.launches or 0 for ex in run.executors)
    # (a loose bound — boxes differ in host speed, 41.8 us was seen at 75 nodes: what it rules out
    # is per-edge or per-segment host work, 10-16 us per segment for the runner)
    assert max(run.host_us) <= max(60.0, 25.0 + 0.5 * nodes), (run.host_us, nodes)
    _check(p, run, store, ids, 0.03)


@gpu
@pytest.mark.timeout(240)
def test_loopback_gpu_device_transport_catches_missing_pull(monkeypatch):
    """Negative control: rank 1 never pulls its received regions (the consumer's wait dropped):
    its consumers read the NaN poison and the check fails."""
    from distributed_llm_scheduler_amd.parallel import devp2p
    monkeypatch.setattr(devp2p, "_TICKS", int(2e8))
    p, ids = _gpu_plan("pipeline", 2)
    store = runtime.make_store(p)

    class _NoPull:
        def wait(self):
            pass

    def drop_pulls(exs):
        comm = exs[1].comm
        orig = comm.irecv

        def irecv(buf, peer, key=None):
            orig(buf, peer, key)  # poisons the region
            return _NoPull()
        comm.irecv = irecv

    run = run_loopback(p, "cuda:0", steps=1, warmup=1, capture=False, store=store, delay_us=200.0,
                       before_steps=drop_pulls, transport="device")
    with pytest.raises(AssertionError):
        _check(p, run, store, ids, 0.03)


@gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 4])
def test_loopback_gpu_device_expert_routed_rows(world, monkeypatch):
    """Expert parallelism over the device transport moves ROUTED ROWS only: each expert GPU
    pulls its experts' token rows (gathered by the device-side routing) and the combine pulls
    each expert's count of compact output rows — far fewer bytes than the fixed-size [M, H]
    edges (expected M*k/E of M rows per expert), no capacity, no host sync, and the logits
    still match fp32 (rows whose router logits nearly tie exempt)."""
    from distributed_llm_scheduler_amd.parallel import devp2p
    from distributed_llm_scheduler_amd.parallel import executor as exm
    monkeypatch.setattr(devp2p, "_TICKS", int(2e9))
    moved = {}
    for routed in (False, True):
        monkeypatch.setattr(exm, "EP_ROUTED", routed)
        p, ids = _gpu_plan("expert", world)
        store = runtime.make_store(p)
        run = run_loopback(p, "cuda:0", steps=1, warmup=1, capture=False, store=store, delay_us=20.0,
                           transport="device")
        assert [ex.comm.errors() for ex in run.executors] == [0] * world
        moved[routed] = sum(ex.comm.bytes_pulled() for ex in run.executors)
        _check(p, run, store, ids, 0.03)
    assert 0 < moved[True] < 0.6 * moved[False], moved


# ------------------------------------------- expert-parallel capacity edges (the RCCL transport)
def test_expert_capacity_edges_planned():
    """BASELINE config 5 (Mixtral-8x7B, 8 requests, DP attention + expert parallelism over 8 GPUs):
    on the RCCL transport the expert edges are capacity messages — ~1.25x the routed rows instead
    of whole [M, H] buffers (round 5: 15.0 GB per step, 4.0x the routed 3.77 GB)."""
    p = runtime.plan("mixtral-8x7b", world=8, seq=512, placement="expert", replicas=8)
    st = p.stats
    assert st["cross_gpu_bytes_rccl"] <= 1.3 * st["cross_gpu_bytes_routed"], st
    assert st["cross_gpu_bytes"] >= 3.9 * st["cross_gpu_bytes_routed"]  # what whole buffers would move
    caps = [i for pr in p.programs for i in pr.instrs if i.rows]
    assert caps and all(i.rows == 160 for i in caps)  # 1.25 x 512 x 2 / 8 rows per expert GPU


@pytest.mark.parametrize("case", ["expert", "expert_dp"])
@pytest.mark.parametrize("cpu_runner", [False, True])
def test_loopback_cpu_expert_capacity_edges(case, cpu_runner):
    """Capacity edges at 4 ranks (one expert per rank, M = 64 rows): every expert edge moves its
    capacity rows (not the [M, H] buffer), the home packs and the expert rank unpacks on the
    device-side routing, and the logits match fp32. (A tiny random router is unbalanced enough
    that some groups overflow 1.25x: those are widened — on both of their ranks — and the step
    re-run; the rest stay capacity edges.)"""
    p, ids = _plan(case, 4, 64)
    caps = {(pr.rank, i.op, i.task, i.peer): i.rows for pr in p.programs for i in pr.instrs if i.rows}
    assert caps and all(r < 64 for r in caps.values())
    store = runtime.make_store(p)
    run = run_loopback(p, "cpu", steps=2, warmup=1, store=store, cpu_runner=cpu_runner)
    tm = {t.id: t for t in p.tasks}
    kept = 0
    for r, st in enumerate(run.stats):
        wide = set(run.ep_widened[r])
        sent = 0
        for i in p.programs[r].instrs:
            if i.op != "send":
                continue
            grp = (i.task if i.experts else tm[i.task].op.inputs[0], i.peer)
            if i.rows and grp not in wide:
                sent += i.rows * tm[i.task].xfer_bytes // 64
                kept += 1
            else:
                sent += tm[i.task].xfer_bytes
        assert st.bytes_sent == sent, (r, st.bytes_sent, sent)
    assert kept > 0, "every capacity edge was widened"
    _check(p, run, store, ids, 0.03)


@pytest.mark.parametrize("world", [2, 4])
def test_loopback_cpu_expert_capacity_overflow_is_exact(world, monkeypatch):
    """Forced overflow: capacities at 0.3x the expected routed rows. The pack / unpack launches
    flag the overflowed groups on both of their ranks, every rank widens them, the job runs the
    step again with whole-buffer edges there, and the logits match fp32 exactly as without
    capacity edges."""
    from distributed_llm_scheduler_amd.parallel import program

    monkeypatch.setattr(program, "EP_CAPACITY", 0.3)
    p, ids = _plan("expert_dp", world, 64)
    assert any(i.rows for pr in p.programs for i in pr.instrs)
    store = runtime.make_store(p)
    run = run_loopback(p, "cpu", steps=1, warmup=1, store=store)
    assert any(run.ep_widened), "0.3x capacities must overflow"
    # a group is widened on both of its ranks
    pairs = {(h, r, peer) for r, ws in enumerate(run.ep_widened) for h, peer in ws}
    assert all((h, peer, r) in pairs for h, r, peer in pairs), pairs
    _check(p, run, store, ids, 0.03)


@gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("factor", [1.25, 0.3])
def test_loopback_gpu_expert_capacity_edges(factor, monkeypatch):
    """Config 5's edges on one MI355X (4 ranks, hub transport = RCCL's p2p semantics, segment
    hipGraphs + native runner, NaN-poisoned receives): capacity messages packed / unpacked by
    the device routing; at 0.3x forced overflow the groups are widened on both ranks and the
    step re-run — the logits match fp32 either way."""
    from distributed_llm_scheduler_amd.parallel import program

    monkeypatch.setattr(program, "EP_CAPACITY", factor)
    p, ids = _gpu_plan("expert_dp", 4)
    assert any(i.rows for pr in p.programs for i in pr.instrs)
    store = runtime.make_store(p)
    run = run_loopback(p, "cuda:0", steps=3, warmup=2, store=store, delay_us=50.0)
    if factor < 1:
        assert any(run.ep_widened)
    _check(p, run, store, ids, 0.03)


# BASELINE configs 3-5 at FULL width through the one-GPU harness (the loopback GPU
# coverage was mini-scale only): one request DAG of GPT-2-medium over 2 ranks under the 8 GB
# reference-cost cap (MRU_spec and EFT: evictions, refills, p2p edges), one full-width Llama-3-8B
# layer tensor-parallel over 2 ranks, one full-width Mixtral-8x7B layer with data-parallel
# attention + expert parallelism over 4 ranks (capacity edges at M = 512). Logits vs fp32.
FULL = {
    "gpt2m_cap_mru": ("gpt2-medium", 2, dict(scheduler="MRU_spec", cap_gb=8.0, replicas=1, cost_model="reference"),
                      ["output_projection"]),
    "gpt2m_cap_eft": ("gpt2-medium", 2, dict(scheduler="EFT", cap_gb=8.0, replicas=1, cost_model="reference"),
                      ["output_projection"]),
    "llama_1l_tp2": ("llama3-8b-1l", 2, dict(placement="tensor", tp=2), ["output_projection"]),
    "mixtral_1l_expert_dp4": ("mixtral-8x7b-1l", 4, dict(placement="expert", replicas=4), "replicas"),
}


@gpu
@pytest.mark.timeout(280)
@pytest.mark.parametrize("case", sorted(FULL))
def test_loopback_gpu_full_width_configs(case):
    model, world, kw, ids = FULL[case]
    p = runtime.plan(model, world=world, seq=512, batch=1, **kw)
    assert p.completed == p.total and _p2p_work(p) > 0
    if ids == "replicas":
        ids = [f"r{k}/output_projection" for k in range(world)]
        assert any(i.rows for pr in p.programs for i in pr.instrs)  # capacity edges at full width
    store = runtime.make_store(p)
    run = run_loopback(p, "cuda:0", steps=2, warmup=2, store=store, delay_us=20.0, autotune=False)
    _check(p, run, store, ids, 0.03)
