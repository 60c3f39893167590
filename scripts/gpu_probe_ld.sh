#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; export DLS_SKIP_BUILD=1
for pad in 0 64 256 1024; do
  for K in 64 768; do
    timeout -k 10 60 python3 benchmarks/probe_gemm_round.py --cfg 34 --K $K --reps 20 --hot --ldpad $pad 2>&1 | grep cfg | sed "s/^/K=$K /" || exit 3
  done
done
