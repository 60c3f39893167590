#!/usr/bin/env python3
"""Per-block error of the GPT-2-small DAG (S = 512) against the fp32 reference, four identical
runs: max |out - ref| / max |ref| of every layer_i_output, in %. The folded norms take their row
statistics from atomics, so the worst element varies from run to run."""
import torch, sys
sys.path.insert(0, "/root/repo")
from distributed_llm_scheduler_amd.parallel import runtime
from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens
from distributed_llm_scheduler_amd.models import reference
S = 512
p = runtime.plan("gpt2", world=1, seq=S, batch=1)
store = runtime.make_store(p)
tok = synthetic_tokens("@tokens", S, p.cfg.vocab_size).view(1, S)
hidden = []
reference.gpt2_forward(p.cfg, store, tok, hidden=hidden)
for rep in range(4):
    ex = runtime.make_executor(p, 0, torch.device("cuda:0"), store, use_graph=False)
    ex.step()
    got = {}
    orig = ex._issue_run
    def issue(i, ins, stats, events, orig=orig, ex=ex):
        orig(i, ins, stats, events)
        tid = ins.task
        if tid.endswith("_output") and tid.startswith("layer_"):
            got[int(tid.split("_")[1])] = ex._views[tid].float().clone()
    ex._issue_run = issue
    ex.step()
    torch.cuda.synchronize()
    errs = []
    for i, ref in enumerate(hidden):
        out = got[i].cpu().view_as(ref)
        errs.append(round((out - ref).abs().max().item() / ref.abs().max().item() * 100, 3))
    print(rep, errs, flush=True)
    del ex
