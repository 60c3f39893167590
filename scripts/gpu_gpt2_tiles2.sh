#!/bin/bash
# Second pass of GPT-2 GEMM tile alternatives (after fc1 -> 25, QKV -> 17), three same-box rounds.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
V=benchmarks/tuning_ab
TAG=g2t2 TABLES="$T0 $V/p2_lm34.json $V/p2_lm35.json $V/p2_op16.json $V/p2_op20.json $V/p2_fc2_16s2.json $V/p2_fc2_20.json $V/p2_qkv16.json $V/p2_qkv20.json $V/p2_fc1_20.json $V/p2_fc1_19.json" ROUNDS=3 bash scripts/gpu_ab_tables.sh || exit 3
