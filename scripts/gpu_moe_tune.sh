#!/bin/bash
# Re-tune Mixtral's grouped expert GEMM shapes (new deep-ring configs) and measure the step.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "grouped or row_range" --timeout 120 --timeout-method thread > gpurun_out/moe_tests.log 2>&1 || { tail -30 gpurun_out/moe_tests.log; exit 3; }
tail -2 gpurun_out/moe_tests.log
timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 10 --warmup 2 > gpurun_out/mix_before.json 2> gpurun_out/mix_before.err || { tail -20 gpurun_out/mix_before.err; exit 4; }
echo "before: $(cut -c1-200 gpurun_out/mix_before.json)"
timeout -k 10 600 python - <<'PY' > gpurun_out/moe_tune.log 2>&1 || { tail -20 gpurun_out/moe_tune.log; exit 5; }
import torch
from distributed_llm_scheduler_amd.ops import tuning
for M, N, K, tg in ((128, 28672, 4096, "sg"), (128, 4096, 14336, "g")):
    best, res = tuning.tune(M, N, K, tg=tg, save=True)
    top = sorted(res.items(), key=lambda kv: kv[1])[:8]
    print(M, N, K, tg, "best", best, "top", [(c, round(t, 1)) for c, t in top], flush=True)
PY
cat gpurun_out/moe_tune.log
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json gpurun_out/gemm_tuning_after.json
timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 10 --warmup 2 > gpurun_out/mix_after.json 2> gpurun_out/mix_after.err || { tail -20 gpurun_out/mix_after.err; exit 6; }
echo "after: $(cut -c1-200 gpurun_out/mix_after.json)"
