#!/bin/bash
# Full GPU check: test suite, smoke, GPT-2 bench + per-dispatch profile.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/r3
export DLS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r3/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || { tail -20 gpurun_out/r3/smoke.log; exit 3; }
tail -1 gpurun_out/r3/smoke.log
OUT=gpurun_out/r3/prof_gpt2 BENCH_ARGS="--no-extras" bash scripts/gpu_prof_gpt2.sh
