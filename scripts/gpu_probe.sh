#!/bin/bash
# Probes: Infinity-Cache pollution by the LM head; kernel trace of the hipGraph GPT-2 step (gaps).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/probe
export DLS_SKIP_BUILD=1
timeout -k 10 300 python benchmarks/bench_mall_step.py > gpurun_out/probe/mall_step.json 2> gpurun_out/probe/mall_step.err || { tail -20 gpurun_out/probe/mall_step.err; exit 3; }
cat gpurun_out/probe/mall_step.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/probe/prof" -o graph -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 > "$ROOT/gpurun_out/probe/prof.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/probe/prof.log"; exit 4; }
tail -1 "$ROOT/gpurun_out/probe/prof.log"
