#!/bin/bash
# GPT-2 fc1 shape (512 x 3072 x 768) under configs 17 / 25 / 22: in-kernel phase stamps.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/stamps
: > gpurun_out/stamps/fc1.txt
for c in 17 25 22 17 25; do timeout -k 5 30 gpubin/gemm_stamps $c 512 3072 768 >> gpurun_out/stamps/fc1.txt 2>&1 || { echo "FAILED $c"; exit 3; }; done
cat gpurun_out/stamps/fc1.txt
