#!/bin/bash
# Configs 42 / 43 (128x96 with more K-tiles in flight): GEMM tests, then in-DAG timing on the
# Llama-3-8B QKV / wo / down shapes against the current choices.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/qkvr; mkdir -p $O
export DLS_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm_shapes or folded_norm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/tuning.json
export DLS_GEMM_TUNING=$O/tuning.json
timeout -k 10 600 python benchmarks/refine_dag.py --model llama3-8b --reps 5 --keys 512x6144x4096,512x4096x4096,512x4096x14336 --cfgs 42,43 > $O/refine.json 2> $O/refine.err || { tail -20 $O/refine.err; exit 5; }
grep -v amdgpu $O/refine.err | tail -25
unset DLS_GEMM_TUNING
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
TAG=mixq TMO=400 STEPS=10 WARM=2 BENCH_ARGS="--model mixtral-8x7b" TABLES="$T0 benchmarks/tuning_ab/qkv_old.json" ROUNDS=2 bash scripts/gpu_ab_tables.sh || exit 6
