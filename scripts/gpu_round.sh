#!/bin/bash
# tests + benches (+ optional cold GEMM landscape) in one call
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
bash scripts/gpu_models.sh || exit $?
if [ -n "$COLD" ]; then bash scripts/gpu_cold.sh || exit $?; fi
if [ -n "$PROF" ]; then MODELS="$PROF" bash scripts/gpu_prof.sh || exit $?; fi
