#!/bin/bash
# Llama-3-8B GEMM tile alternatives against the shipped table, two alternating same-box rounds.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
V=benchmarks/tuning_ab
TAG=llt TMO=300 STEPS=20 WARM=3 BENCH_ARGS="--model llama3-8b" TABLES="$T0 $V/wo_14.json $V/wo_10.json $V/down_0.json $V/down_10.json $V/lml_13.json $V/gu_13.json" ROUNDS=2 bash scripts/gpu_ab_tables.sh || exit 3
