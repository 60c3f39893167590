#!/bin/bash
# GPT-2 GEMM tile alternatives, each against the shipped table, three alternating same-box rounds.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
V=benchmarks/tuning_ab
TAG=g2t TABLES="$T0 $V/qkv_25.json $V/qkv_17.json $V/qkv_26.json $V/op_17.json $V/op_24.json $V/fc2_24.json" ROUNDS=3 bash scripts/gpu_ab_tables.sh || exit 3
