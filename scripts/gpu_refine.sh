#!/bin/bash
# Whole-step GEMM config refinement for each model, then a clean bench with the refined table.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
for m in ${MODELS:-gpt2 llama3-8b mixtral-8x7b}; do
  echo "== refine $m"
  timeout -k 10 900 python bench.py --model "$m" --steps 10 --warmup 2 --refine-tuning > "gpurun_out/refine_$m.out" 2> "gpurun_out/refine_$m.err" || { tail -20 "gpurun_out/refine_$m.err"; exit 3; }
  grep "refinement" "gpurun_out/refine_$m.err" | cut -c1-1500
  cut -c1-200 "gpurun_out/refine_$m.out"
done
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json gpurun_out/
