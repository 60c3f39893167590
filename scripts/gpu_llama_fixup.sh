#!/bin/bash
# Llama-3-8B: post-norm split-K reduces (wo, down) vs the in-launch combine with the norm folded
# into the consumer GEMM (row statistics handed over), alternating same-box runs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
TAG=llfix TMO=300 STEPS=20 WARM=3 BENCH_ARGS="--model llama3-8b" TABLES="$T0 $T0@DLS_HANDOFF_MAX_K=4096 $T0@DLS_FIXUP_MAX_KB=512 $T0@DLS_FIXUP_MAX_KB=512,DLS_HANDOFF_MAX_K=4096" ROUNDS=2 bash scripts/gpu_ab_tables.sh || exit 3
