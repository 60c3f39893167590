#!/bin/bash
# Config 42 (192x256 expert tiles): grouped-GEMM tests and the Mixtral grouped probe.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/moe42
export DLS_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "grouped or gemm_shapes" --timeout 120 --timeout-method thread > gpurun_out/moe42/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/moe42/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_grouped.py 128,28672,4096,s 128,4096,14336 > gpurun_out/moe42/grouped.log 2>&1 || { tail -20 gpurun_out/moe42/grouped.log; exit 4; }
grep '^{' gpurun_out/moe42/grouped.log
