#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 900 python benchmarks/bench_cold_gemm.py --shapes "${SHAPES:-all}" > gpurun_out/cold_gemm.jsonl 2> gpurun_out/cold_gemm.err || { tail -20 gpurun_out/cold_gemm.err; exit 3; }
cat gpurun_out/cold_gemm.jsonl
