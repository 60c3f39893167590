#!/bin/bash
# A/B of an executor switch in one box: bench each model with VAR=0 and VAR=1, alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
VAR=${VAR:-DLS_STATS_HANDOFF}
for m in ${MODELS:-gpt2 llama3-8b}; do
  for rep in 1 2; do
    for v in 0 1; do
      out=$(env $VAR=$v timeout -k 10 600 python bench.py --model "$m" --steps ${STEPS:-20} --warmup 3 2> gpurun_out/ab_err.log) || { tail -5 gpurun_out/ab_err.log; exit 3; }
      echo "$m $VAR=$v rep$rep $(echo "$out" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
