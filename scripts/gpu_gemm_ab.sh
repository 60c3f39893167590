#!/bin/bash
# GEMM numerics + microbenchmarks after a kernel change: GPU tests, K-sweep, launch floor.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_gemm_ksweep.py > gpurun_out/ksweep.log 2>&1 || { tail -5 gpurun_out/ksweep.log; exit 4; }
cat gpurun_out/ksweep.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 5; }
cat gpurun_out/bench1.json
