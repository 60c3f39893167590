"""Device-initiated p2p transport (parallel/devp2p.py): message slots and source regions from
the plan alone (CPU), and a process-per-rank job whose ranks map each other's arenas and
mailboxes through IPC handles (GPU: two processes sharing the one MI355X of the box; the
in-process form runs in tests/test_loopback.py)."""
import os
import socket

import pytest
import torch

from distributed_llm_scheduler_amd.parallel import runtime
from distributed_llm_scheduler_amd.parallel.devp2p import edge_slots, source_regions


@pytest.mark.parametrize("kw", [dict(placement="pipeline", replicas=2), dict(placement="tensor", tp=2),
                                dict(placement="sequence", sp=2), dict(replicas=2, cap_gb=0.0001)])
def test_slots_pair_every_send_with_its_recv(kw):
    """Every send / psend gets one slot; every recv and peer load of the consumer finds the
    producer's slot and a source region as large as its own receive region."""
    model = "tiny-llama" if kw.get("placement") == "tensor" else "tiny-gpt2"
    p = runtime.plan(model, world=2, seq=32, **kw)
    slots, src = edge_slots(p.programs), source_regions(p.programs, p.param_bytes)
    assert set(slots) == set(src) and sorted(slots.values()) == list(range(len(slots)))
    n_recv = 0
    for pr in p.programs:
        for ins in pr.instrs:
            if ins.op == "recv":
                key = (ins.peer, pr.rank, ("act", ins.task))
                assert key in slots
                assert src[key][2] == pr.act_bytes[ins.task]
                n_recv += 1
            elif ins.op == "load" and ins.peer >= 0:
                assert (ins.peer, pr.rank, ("param", ins.param, ins.gpos)) in slots
                n_recv += 1
    assert n_recv == len(slots) > 0


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ipc_worker(rank, world, port, q):
    import torch.distributed as dist

    from distributed_llm_scheduler_amd.models import reference
    from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")  # both ranks on the box's one GPU, separate processes
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # only for the handle exchange
    try:
        p = runtime.plan("mini-gpt2", world=world, seq=64, batch=2, placement="pipeline", replicas=2)
        store = runtime.make_store(p)
        pg = runtime.p2p_group(p, rank, dev, dist.group.WORLD, transport="device")
        ex = runtime.make_executor(p, rank, dev, store, pg=pg, autotune=False)
        for _ in range(2):
            ex.step()
        torch.cuda.synchronize()
        dist.barrier()
        ex.comm.reset_errors()
        assert ex.capture()
        for _ in range(5):
            ex.step()
        torch.cuda.synchronize()
        res = {"rank": rank, "err": ex.comm.errors(), "graph": ex._graph_exec is not None, "checks": []}
        for k in range(2):
            tid = f"r{k}/output_projection"
            if p.owner(tid) == rank:
                out = ex.output(tid).float().cpu()
                B, S = out.shape[0], out.shape[1]
                tok = synthetic_tokens(f"r{k}/@tokens", B * S, p.cfg.vocab_size).view(B, S)
                ref = reference.forward(p.cfg, store, tok)
                res["checks"].append(((out - ref).abs().max().item(), ref.abs().max().item()))
        dist.barrier()
        q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.isolated
@pytest.mark.timeout(240)
def test_device_transport_across_processes_via_ipc():
    """Two rank PROCESSES on one MI355X: arenas and mailboxes exchanged as IPC handles, edges
    pulled by kernels, each rank's step one hipGraph; no wait timed out, logits match fp32."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_ipc_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=200)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    res = sorted((q.get(timeout=5) for _ in range(2)), key=lambda r: r["rank"])
    assert [r["err"] for r in res] == [0, 0] and all(r["graph"] for r in res)
    checks = [c for r in res for c in r["checks"]]
    assert len(checks) == 2
    for err, scale in checks:
        assert err < 0.03 * scale, (err, scale)


@pytest.mark.gpu
@pytest.mark.isolated
@pytest.mark.timeout(120)
def test_batched_notify_kernel():
    """The sends of one program point notify from ONE launch (p2p_notify_many): every consumer
    flag carries the producer's step, step after step."""
    from distributed_llm_scheduler_amd import ops
    from distributed_llm_scheduler_amd.parallel.devp2p import Mailbox

    e = ops.ext()
    dev = torch.device("cuda:0")
    n = 5
    cons, prod = Mailbox(n, dev), Mailbox(n, dev)
    for step in (1, 2, 3):
        e.p2p_tick(prod.step)
        e.p2p_notify_many([cons.ready_addr(cons.base, k) for k in range(n)], prod.step)
        torch.cuda.synchronize()
        assert cons.ready.tolist() == [step] * n
