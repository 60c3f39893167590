#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" > gpurun_out/pytest_gemm.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gemm.log
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_gemm.log | head -20; exit $rc; }
timeout -k 10 500 python benchmarks/bench_kernels.py --only gemm > gpurun_out/kbench_gemm.jsonl 2> gpurun_out/kbench_gemm.err; rc=$?
cat gpurun_out/kbench_gemm.jsonl; tail -3 gpurun_out/kbench_gemm.err; exit $rc
