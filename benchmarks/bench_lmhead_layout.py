import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from distributed_llm_scheduler_amd import ops
from distributed_llm_scheduler_amd.ops.tuning import _graph_time
ext = ops.ext()
for M, N in ((50304, 512), (512, 50304)):
    for cfg in (0, 1, 8, 12, 13, 14):
        row = {"M": M, "N": N, "cfg": cfg}
        for K in (64, 768):
            x = torch.randn(M, K, device="cuda").bfloat16()
            w = torch.randn(N, K, device="cuda").bfloat16()
            o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row[K] = round(_graph_time(lambda i: ext.gemm(x, w, None, None, 0, 1.0, o, cfg, 1), reps=20), 2)
        print(json.dumps(row), flush=True)
    row = {"M": M, "N": N, "cfg": "torch"}
    for K in (64, 768):
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = torch.randn(N, K, device="cuda").bfloat16()
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        row[K] = round(_graph_time(lambda i: torch.matmul(x, w.t(), out=o), reps=20), 2)
    print(json.dumps(row), flush=True)
