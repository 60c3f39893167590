#!/bin/bash
# Round-3 A/B on the fixed build: GPT-2 LM-head config, Llama-3-8B new tile configs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
TAG=gpt2c TABLES="$T0 benchmarks/tuning_ab/lm34.json" ROUNDS=3 bash scripts/gpu_ab_tables.sh || exit 3
TAG=llamac TMO=300 STEPS=20 WARM=3 BENCH_ARGS="--model llama3-8b" TABLES="$T0 benchmarks/tuning_ab/gu37.json benchmarks/tuning_ab/gu37_qkv38.json benchmarks/tuning_ab/gu37_qkv38_wo40.json" ROUNDS=2 bash scripts/gpu_ab_tables.sh || exit 4
