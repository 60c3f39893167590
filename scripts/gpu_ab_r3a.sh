#!/bin/bash
# Round-3 A/B: GPT-2 LM-head config (13 vs 34 vs 35), HIP kernel arguments in device memory,
# Llama-3-8B new tile configs and the K=4096 statistics hand-off.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
T0=distributed_llm_scheduler_amd/ops/gemm_tuning.json
TAG=gpt2 TABLES="$T0 benchmarks/tuning_ab/lm34.json benchmarks/tuning_ab/lm35.json $T0@HIP_FORCE_DEV_KERNARG=1 $T0@HIP_FORCE_DEV_KERNARG=0" ROUNDS=3 bash scripts/gpu_ab_tables.sh || exit 3
TAG=llama TMO=300 STEPS=20 WARM=3 BENCH_ARGS="--model llama3-8b" TABLES="$T0 benchmarks/tuning_ab/gu37.json benchmarks/tuning_ab/gu37_qkv38.json benchmarks/tuning_ab/gu37_qkv38_wo40.json benchmarks/tuning_ab/gu37_qkv38_wo40.json@DLS_HANDOFF_MAX_K=4096" ROUNDS=2 bash scripts/gpu_ab_tables.sh || exit 4
