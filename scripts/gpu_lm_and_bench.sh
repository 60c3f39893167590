#!/bin/bash
# LM-head configs microbenchmark, then the GPT-2 bench + per-dispatch profile.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 200 python benchmarks/bench_lmhead.py --cfgs 34,35,8,9,12,13,10 --json gpurun_out/lmhead2.json > gpurun_out/lmhead2.log 2>&1 || { tail -20 gpurun_out/lmhead2.log; exit 4; }
grep -v amdgpu.ids gpurun_out/lmhead2.log
OUT=gpurun_out/prof_gpt2b BENCH_ARGS="--no-extras" bash scripts/gpu_prof_gpt2.sh
