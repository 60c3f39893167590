"""Per-layer routed rows of Mixtral-8x7B's benchmarked step (batch 1 x 512 tokens, top-2 of 8
experts): the count of rows each expert gets in every MoE layer, from the device routing of a
real step (are the slow expert launches the layers whose busiest expert
exceeds one row tile?). Writes JSON {layer: [rows per expert]}."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_scheduler_amd.parallel import runtime  # noqa: E402

out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mixtral_rows.json"
p = runtime.plan("mixtral-8x7b", world=1, seq=512, batch=1)
ex = runtime.make_executor(p, 0, torch.device("cuda:0"), runtime.make_store(p, device_init=True), use_graph=False)
ex.step()
ex.step()
torch.cuda.synchronize()
rows = {}
for key, r in ex._moe_memo.items():
    if key[0] != "route":
        continue
    off = r[4].cpu().tolist()
    layer = int(key[1].split("_")[1])
    rows[layer] = [off[e + 1] - off[e] for e in range(len(off) - 1)]
os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
json.dump({str(k): v for k, v in sorted(rows.items())}, open(out_path, "w"))
for k, v in sorted(rows.items()):
    print(k, max(v), min(v), v)
