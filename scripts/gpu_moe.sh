#!/bin/bash
# MoE path: routing / grouped-GEMM / executor tests, Mixtral-8x7B bench, per-step kernel breakdown.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/moe
export DLS_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_executor_gpu.py -k "moe or grouped or mixtral or expert" > gpurun_out/moe/tests.log 2>&1 || { tail -30 gpurun_out/moe/tests.log; exit 3; }
tail -2 gpurun_out/moe/tests.log
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 10 --warmup 3 > gpurun_out/moe/bench.json 2> gpurun_out/moe/bench.err || { tail -20 gpurun_out/moe/bench.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/moe/bench.json')); print('mixtral', d['value'], 'ms')"
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/moe/prof" -o mixtral -- \
    python3 "$ROOT/bench.py" --model mixtral-8x7b --steps 3 --warmup 2 --no-graph > "$ROOT/gpurun_out/moe/prof.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/moe/prof.log"; exit 5; }
  cd "$ROOT" && python tools/analyze_trace.py gpurun_out/moe/prof/mixtral_kernel_trace.csv --steps 2 > gpurun_out/moe/breakdown.txt && head -24 gpurun_out/moe/breakdown.txt
fi
