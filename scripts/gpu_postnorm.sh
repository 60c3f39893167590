#!/bin/bash
# Post-norm fusion: kernel + executor tests, then Llama-3-8B / Mixtral A/B of DLS_POST_NORM.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/pn
export DLS_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_executor_gpu.py -k "post_norm or moe or grouped or dag_on_gpu" > gpurun_out/pn/tests.log 2>&1 || { tail -30 gpurun_out/pn/tests.log; exit 3; }
tail -2 gpurun_out/pn/tests.log
for m in llama3-8b mixtral-8x7b; do
  for i in 1 2; do
    for v in 0 1; do
      DLS_POST_NORM=$v timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 3 > gpurun_out/pn/ab.json 2> gpurun_out/pn/ab.err || { tail -5 gpurun_out/pn/ab.err; exit 4; }
      echo "$m DLS_POST_NORM=$v $(python -c 'import json;print(json.load(open("gpurun_out/pn/ab.json"))["ms_per_step"])')"
    done
  done
done
