#!/bin/bash
# A/B of an environment switch on the GPT-2 bench: alternating runs, 3 each.
# usage: VAR=DLS_SPLITK_FIXUP A=0 B=1 bash scripts/gpu_ab_env.sh
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
for i in 1 2 3; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --steps 200 --warmup 10 ${BENCH_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 3; }
    echo "$VAR=$v $(python -c 'import json;print(json.load(open("gpurun_out/ab.json"))["ms_per_step"])')"
  done
done
