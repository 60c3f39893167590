#!/usr/bin/env python3
"""Per-row error of one full-width Mixtral layer DAG vs the fp32 reference (debug aid):
prints rows whose error exceeds 3 % of the logit scale and their router margins."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_scheduler_amd.models import reference  # noqa: E402
from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402
from distributed_llm_scheduler_amd.parallel.executor import synthetic_tokens  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "mixtral-8x7b-1l"
seq = int(sys.argv[2]) if len(sys.argv) > 2 else 512
graph = len(sys.argv) > 3 and sys.argv[3] == "graph"
p = runtime.plan(model, world=1, seq=seq, batch=1)
store = runtime.make_store(p)
ex = runtime.make_executor(p, 0, torch.device("cuda:0"), store, use_graph=graph)
ex.step()
if graph:
    ex.capture()
    ex.step()
torch.cuda.synchronize()
out = ex.output("output_projection").float().cpu()
tok = synthetic_tokens("@tokens", seq, p.cfg.vocab_size).view(1, seq)
margins = []
ref = reference.forward(p.cfg, store, tok, router_margins=margins)
scale = ref.abs().max().item()
row_err = (out - ref).abs().amax(-1)[0]
bad = (row_err > 0.03 * scale).nonzero().flatten().tolist()
env = {k: v for k, v in os.environ.items() if k.startswith("DLS_")}
print(f"{model} S={seq} graph={graph} env={env}: bad rows {bad[:20]} (of {seq}); max err {row_err.max():.4f} "
      f"scale {scale:.3f}; margins of bad rows {[round(float(m[0, r]), 4) for m in margins for r in bad[:5]]}",
      flush=True)
