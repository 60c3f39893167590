#!/bin/bash
# In-kernel phase stamps of the GPT-2 GEMM shapes (benchmarks/gemm_stamps.hip, prebuilt in gpubin/).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/stamps
run() { timeout -k 5 30 gpubin/gemm_stamps "$@" >> gpurun_out/stamps/stamps.txt 2>&1 || { echo "FAILED $*"; exit 3; }; }
: > gpurun_out/stamps/stamps.txt
run 24 512 2304 768
run 27 512 768 768
run 27 512 768 3072
run 17 512 3072 768
run 24 512 768 3072
run 34 512 50304 768
cat gpurun_out/stamps/stamps.txt
