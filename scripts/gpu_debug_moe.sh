#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; export DLS_SKIP_BUILD=1
run() { timeout -k 10 120 env "$@" python benchmarks/debug_mixtral_rows.py mixtral-8x7b-1l 512 2>&1 | grep -v amdgpu.ids | tail -2 || exit 3; }
run DLS_X=0
run DLS_POST_NORM=0
run DLS_MOE_FUSED_ROUTE=0
run DLS_MOE_BATCH=0
run DLS_EXPERT_NT=0
timeout -k 10 120 python benchmarks/debug_mixtral_rows.py mixtral-8x7b-1l 512 graph 2>&1 | grep -v amdgpu.ids | tail -1
timeout -k 10 120 env DLS_GEMM_TUNING=/nonexistent python benchmarks/debug_mixtral_rows.py mixtral-8x7b-1l 512 2>&1 | grep -v amdgpu.ids | tail -1
