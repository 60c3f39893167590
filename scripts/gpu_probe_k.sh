#!/bin/bash
# One-round GEMM time vs K (hot operands): slope = main loop per K-tile, intercept = prologue + epilogue.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/probe
export DLS_SKIP_BUILD=1
for c in 34 10 ${EXTRA_CFGS}; do
  bn=256; [ $c = 10 ] && bn=128
  for K in 64 128 256 768 1536 3072; do
    timeout -k 10 60 python3 benchmarks/probe_gemm_round.py --cfg $c --bn $bn --K $K --reps 20 ${MODE} 2>&1 | grep cfg | sed "s/^/K=$K /" || exit 3
  done
done
