"""Sequence (context) parallelism as a DAG transform (models/transforms.py
``sequence_parallel``): chunked token-wise nodes, per-chunk QKV nodes and chunk-vs-prefix
attention nodes. Checked on the CPU fake-device executor against the unchunked reference
forward — single rank and two gloo ranks with the chunks on different devices (the K/V
edges between chunks are then point-to-point transfers)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_scheduler_amd.models import reference, registry
from distributed_llm_scheduler_amd.parallel import runtime
from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens


def _logits(p, ex, P):
    outs = [ex.output(f"output_projection.sp{c}").float() for c in range(P)]
    return torch.cat(outs, dim=1)


def _ref(p, store, B, S):
    tok = synthetic_tokens("@tokens", B * S, p.cfg.vocab_size).view(B, S)
    return reference.forward(p.cfg, store, tok)


def test_transform_structure():
    tasks, groups, cfg = registry.build("tiny-gpt2", seq=32, sp=4)
    base, _, _ = registry.build("tiny-gpt2", seq=32)
    ids = {t.id for t in tasks}
    n_attn = sum(1 for t in base if t.op.kind == "attention")
    # every non-attention node x4, every attention node -> 4 qkv + 4 attention chunks
    assert len(tasks) == 4 * (len(base) - n_attn) + 8 * n_attn
    a3 = next(t for t in tasks if t.id == "layer_0_attention.sp3")
    assert a3.op.kind == "attn_sp" and a3.dependencies == [f"layer_0_attention.qkv.sp{j}" for j in range(4)]
    a0 = next(t for t in tasks if t.id == "layer_0_attention.sp0")
    assert a0.dependencies == ["layer_0_attention.qkv.sp0"]
    assert all(d in ids for t in tasks for d in t.dependencies)
    emb = next(t for t in tasks if t.id == "embedding.sp2")
    assert emb.op.inputs == ["@tokens"] and emb.op.attrs["seq_chunk"] == (2, 4)
    with pytest.raises(ValueError):
        registry.build("tiny-gpt2", seq=30, sp=4)


@pytest.mark.parametrize("model,P,B", [("tiny-gpt2", 2, 1), ("tiny-gpt2", 4, 2), ("tiny-llama", 2, 1),
                                       ("tiny-llama", 4, 1)])
def test_single_rank_matches_reference(model, P, B):
    S = 32
    p = runtime.plan(model, world=1, seq=S, batch=B, sp=P)
    assert p.completed == p.total
    store = runtime.make_store(p)
    ex = runtime.make_executor(p, 0, "cpu", store)
    ex.step()
    out = _logits(p, ex, P)
    ref = _ref(p, store, B, S)
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() < 0.02 * ref.abs().max().item()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, model, P, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        S = 32
        p = runtime.plan(model, world=world, seq=S, batch=1, sp=P, placement="sequence")
        store = runtime.make_store(p)
        ex = runtime.make_executor(p, rank, "cpu", store, pg=dist.group.WORLD)
        for _ in range(2):
            st = ex.step()
        mine = {c: ex.output(f"output_projection.sp{c}").float() for c in range(P)
                if p.placement.get(f"output_projection.sp{c}") == rank}
        ref = _ref(p, store, 1, S)
        Sc = S // P
        errs = [((o - ref[:, c * Sc:(c + 1) * Sc]).abs().max().item(), ref.abs().max().item())
                for c, o in mine.items()]
        q.put({"rank": rank, "sends": st.sends, "recvs": st.recvs, "errs": errs})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["tiny-gpt2", "tiny-llama"])
def test_two_ranks_sequence_placement(model):
    world, P = 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, P, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(timeout=240)
    assert all(pr.exitcode == 0 for pr in procs), [pr.exitcode for pr in procs]
    res = sorted([q.get(timeout=5) for _ in range(world)], key=lambda r: r["rank"])
    # chunk 0's K/V travel to the rank holding chunk 1 (one edge per layer)
    assert res[0]["sends"] > 0 and res[1]["recvs"] > 0
    errs = [e for r in res for e in r["errs"]]
    assert len(errs) == P
    for err, scale in errs:
        assert err < 0.02 * scale
