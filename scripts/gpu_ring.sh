#!/bin/bash
# Ring-mainloop GEMM: numerics tests for the new configs, then the LM-head benchmark.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "(test_gemm_shapes and (-34- or -35- or -98-)) or (row_stats and 34) or (external_stats and (34 or 35))" \
  > gpurun_out/ring_tests.log 2>&1; rc=$?
tail -5 gpurun_out/ring_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_lmhead.py --json gpurun_out/lmhead1.json > gpurun_out/lmhead1.log 2>&1 || { tail -20 gpurun_out/lmhead1.log; exit 4; }
grep -v amdgpu.ids gpurun_out/lmhead1.log
