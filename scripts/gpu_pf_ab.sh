#!/bin/bash
# Epilogue-operand prefetch build: GEMM / executor GPU tests, then a same-box A/B against the
# tree in ./abtree (the build without it), both on this tree's tuning table.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/pf
export DLS_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pf/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pf/pytest.log; [ $rc -eq 0 ] || exit $rc
export DLS_GEMM_TUNING="$ROOT/distributed_llm_scheduler_amd/ops/gemm_tuning.json"
ALT=abtree ROUNDS=4 BENCH_ARGS="--no-extras" bash scripts/gpu_ab_trees.sh | tee gpurun_out/pf/ab_gpt2.txt || exit 4
