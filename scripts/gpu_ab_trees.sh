#!/bin/bash
# A/B of two source trees' bench.py on one box (alternating runs): $ALT (another tree, built
# in-tree) against this tree.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/abt
export DLS_SKIP_BUILD=1
for i in $(seq ${ROUNDS:-3}); do
  for t in ${ORDER:-"$ALT" .}; do
    timeout -k 10 200 python "$t/bench.py" --steps 200 --warmup 10 ${BENCH_ARGS:-} > gpurun_out/abt/r.json 2> gpurun_out/abt/r.err || { tail -5 gpurun_out/abt/r.err; exit 3; }
    echo "$t $(python -c 'import json;print(json.load(open("gpurun_out/abt/r.json"))["ms_per_step"])')"
  done
done
