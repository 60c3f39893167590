#!/bin/bash
# rocprofv3 kernel stats of bench.py for each model in $MODELS (default llama3-8b mixtral-8x7b).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/prof
export DLS_SKIP_BUILD=1
cd /tmp && export TMPDIR=/tmp
for m in ${MODELS:-llama3-8b mixtral-8x7b}; do
  echo "== $m"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o "$m" -- \
    python3 "$ROOT/bench.py" --model "$m" --steps 5 --warmup 2 --no-graph ${BENCH_ARGS:-} > "$ROOT/gpurun_out/prof_$m.log" 2>&1 \
    || { tail -20 "$ROOT/gpurun_out/prof_$m.log"; exit 7; }
  head -25 "$ROOT/gpurun_out/prof/${m}_kernel_stats.csv" | cut -d, -f1-8 | cut -c1-220
done
