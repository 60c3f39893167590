#!/bin/bash
# Same-box A/B of this tree's GPT-2 headline against another tree ($ALT, built in-tree;
# default: the round's starting tree in ./abtree), alternating runs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/abh
export DLS_SKIP_BUILD=1
ALT=${ALT:-abtree}
for i in $(seq ${ROUNDS:-3}); do
  for t in "$ALT" .; do
    extra=""; [ "$t" = "." ] && extra="--no-extras"
    timeout -k 10 200 python "$t/bench.py" --steps 200 --warmup 10 $extra ${BENCH_ARGS:-} > gpurun_out/abh/r.json 2> gpurun_out/abh/r.err || { tail -5 gpurun_out/abh/r.err; exit 3; }
    echo "$t $(python -c 'import json;print(json.load(open("gpurun_out/abh/r.json"))["ms_per_step"])')"
  done
done
