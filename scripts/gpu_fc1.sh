#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
bash scripts/gpu_stamps_fc1.sh || exit 3
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
TAG=fc1 TABLES="$T0 benchmarks/tuning_ab/fc1_25.json benchmarks/tuning_ab/fc1_22.json" ROUNDS=3 bash scripts/gpu_ab_tables.sh || exit 4
