#!/bin/bash
# Exhaustive in-DAG GEMM refinement of the GPT-2 step, then an A/B bench: original table vs refined.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/tune
export DLS_SKIP_BUILD=1
MODEL=${MODEL:-gpt2}
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json gpurun_out/tune/orig.json
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json gpurun_out/tune/refined.json
DLS_GEMM_TUNING=gpurun_out/tune/orig.json timeout -k 10 200 python bench.py --model $MODEL --steps 100 --warmup 5 > gpurun_out/tune/bench_orig0.json 2>/dev/null || exit 3
DLS_GEMM_TUNING=gpurun_out/tune/refined.json timeout -k 10 900 python benchmarks/refine_dag.py --model $MODEL --reps ${REPS:-20} > gpurun_out/tune/refine.json 2> gpurun_out/tune/refine.err || { tail -20 gpurun_out/tune/refine.err; exit 4; }
for i in 1 2; do
  DLS_GEMM_TUNING=gpurun_out/tune/refined.json timeout -k 10 200 python bench.py --model $MODEL --steps 100 --warmup 5 > gpurun_out/tune/bench_refined$i.json 2>/dev/null || exit 5
  DLS_GEMM_TUNING=gpurun_out/tune/orig.json timeout -k 10 200 python bench.py --model $MODEL --steps 100 --warmup 5 > gpurun_out/tune/bench_orig$i.json 2>/dev/null || exit 6
done
for f in gpurun_out/tune/bench_*.json; do python -c "import json,sys; print(sys.argv[1], json.load(open(sys.argv[1]))['value'])" $f; done
