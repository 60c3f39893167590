#!/bin/bash
# Kernel microbenchmarks (ours vs torch library paths) on one MI355X.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 500 python benchmarks/bench_kernels.py "$@" > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.err; rc=$?
cat gpurun_out/kbench.jsonl; tail -5 gpurun_out/kbench.err; exit $rc
