#!/usr/bin/env python3
"""BASELINE.json's multi-GPU configurations at FULL model size on ONE MI355X, through the
single-GPU loopback harness (parallel/loopback.py): every rank of the N-rank job is a real
executor with its own stream and host thread, the cross-GPU DAG edges go through the loopback
hub with RCCL's p2p semantics (copies on a hub stream, stream-side waits), programs with p2p
replay from segment hipGraphs + the native step runner. What this shows: the multi-GPU programs
of these configs run end to end on the device and (for the full-width one-layer variants) match
the fp32 reference. What it does not show: xGMI time — the ranks share one GPU, so a step costs
the SUM of the ranks' work.

    python benchmarks/loopback_configs.py [--configs gpt2m_cap,llama_pipeline,mixtral_expert] [--check]

  gpt2m_cap       GPT-2-medium, ONE request DAG over 2 ranks, MRU_spec under an 8 GB/GPU cap
                  (reference cost model: evictions + refills), BASELINE config 3
  llama_pipeline  Llama-3-8B, 8 micro-batches, layer blocks pipelined over 8 ranks, config 4
  mixtral_expert  Mixtral-8x7B, expert e on rank e % 8, the rest of the layer on rank 0, config 5
"""
import argparse
import json
import os
import sys
import time

import torch

os.environ["GPU_MAX_HW_QUEUES"] = "32"  # 8 ranks' streams in this process (parallel/loopback.py)
TRANSPORT = "hub"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402
from distributed_llm_scheduler_amd.parallel.loopback import run_loopback  # noqa: E402

CONFIGS = {
    "gpt2m_cap": dict(model="gpt2-medium", world=2, scheduler="MRU_spec", cap_gb=8.0, replicas=1,
                      cost_model="reference"),
    # the same cap placed by EFT's steady-state partition (one pipeline stage per GPU)
    "gpt2m_cap_eft": dict(model="gpt2-medium", world=2, scheduler="EFT", cap_gb=8.0, replicas=1,
                          cost_model="reference"),
    "llama_pipeline": dict(model="llama3-8b", world=8, placement="pipeline", replicas=8),
    # one request per GPU (data-parallel attention) with the experts spread over the 8 GPUs
    "mixtral_expert": dict(model="mixtral-8x7b", world=8, placement="expert", replicas=8),
}
# full-width one-layer variants whose fp32 reference forward fits a CPU check
# (a one-layer model has no pipeline stages to split: its check runs the layer tensor-parallel)
CHECK = {"llama_pipeline": dict(model="llama3-8b-1l", world=2, placement="tensor", tp=2),
         "mixtral_expert": dict(model="mixtral-8x7b-1l", world=8, placement="expert", replicas=1),
         "gpt2m_cap_eft": dict(model="gpt2-medium", world=2, scheduler="EFT", cap_gb=8.0, replicas=1,
                               cost_model="reference"),
         "gpt2m_cap": dict(model="gpt2-medium", world=2, scheduler="MRU_spec", cap_gb=8.0, replicas=1,
                           cost_model="reference")}


def run(name, kw, steps, check):
    kw = dict(kw)
    model, world = kw.pop("model"), kw.pop("world")
    t0 = time.time()
    p = runtime.plan(model, world=world, seq=512, batch=1, **kw)
    store = runtime.make_store(p, device_init=not check and all(runtime.device_init_ok(p, r) for r in range(world)))
    res = run_loopback(p, "cuda:0", steps=steps, warmup=2, store=store, delay_us=0.0, poison=False, autotune=True,
                       transport=TRANSPORT)
    out = {"config": name, "model": model, "world": world, "tasks_completed": p.completed, "tasks_total": p.total,
           "cross_gpu_edges": p.stats["cross_gpu_edges"], "cross_gpu_mb": round(p.stats["cross_gpu_bytes"] / 1e6, 2),
           "cross_gpu_mb_routed": round(p.stats["cross_gpu_bytes_routed"] / 1e6, 2), "transport": TRANSPORT,
           "issue_modes": res.issue_modes,
           "transfers_total": res.hub.transfers if res.hub is not None else None,
           "pulled_mb_last_steps": (round(sum(ex.comm.bytes_pulled() for ex in res.executors) / 1e6, 2)
                                    if TRANSPORT == "device" else None),
           "host_us_per_step": [round(h, 1) for h in res.host_us],
           "ms_per_step_all_ranks_on_one_gpu": round(max(res.step_ms), 3), "wall_s": round(time.time() - t0, 1)}
    if check:
        from distributed_llm_scheduler_amd.models import reference
        from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens
        errs = []
        for t in p.tasks:
            if t.op is not None and t.op.kind == "lm_head" and t.id in p.placement:
                rid = t.id.split("/")[0] + "/" if "/" in t.id else ""
                o = res.executors[p.placement[t.id]].output(t.id).float().cpu()
                tok = synthetic_tokens(f"{rid}@tokens", o.shape[0] * o.shape[1], p.cfg.vocab_size).view(o.shape[0], -1)
                margins = []
                ref = reference.forward(p.cfg, store, tok, router_margins=margins)
                row = (o - ref).abs().amax(-1) / ref.abs().max()
                if margins:  # MoE near-tie rows may legitimately route differently under bf16
                    row = row[~torch.stack([m.abs() < 0.05 for m in margins]).any(0)]
                errs.append(round(row.max().item(), 4))
        out["max_rel_err_vs_fp32"] = errs
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="gpt2m_cap,llama_pipeline,mixtral_expert")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--check", action="store_true", help="full-width one-layer variants, compared with fp32")
    ap.add_argument("--transport", default="hub", choices=["hub", "device"],
                    help="hub: RCCL semantics through the loopback hub; device: edges moved by kernels "
                         "(parallel/devp2p.py), each rank's step one hipGraph")
    a = ap.parse_args()
    global TRANSPORT
    TRANSPORT = a.transport
    for name in a.configs.split(","):
        run(name, (CHECK if a.check else CONFIGS)[name], a.steps, a.check)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
