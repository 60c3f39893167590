#!/bin/bash
# Llama-3-8B per-step kernel breakdown with and without the post-norm fusion.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/pnprof
export DLS_SKIP_BUILD=1
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  DLS_POST_NORM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pnprof/p$v" -o llama -- \
    python3 "$ROOT/bench.py" --model llama3-8b --steps 3 --warmup 2 --no-graph > "$ROOT/gpurun_out/pnprof/p$v.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/pnprof/p$v.log"; exit 5; }
  (cd "$ROOT" && python tools/analyze_trace.py gpurun_out/pnprof/p$v/llama_kernel_trace.csv --steps 2 > gpurun_out/pnprof/breakdown_$v.txt && head -16 gpurun_out/pnprof/breakdown_$v.txt)
done
