#!/bin/bash
# Mixtral A/B/C of DLS_POST_NORM (off / every producer / residual GEMMs only) + kernel breakdown.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/pn
export DLS_SKIP_BUILD=1
for i in 1 2; do
  for v in 0 1 gemm; do
    DLS_POST_NORM=$v timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 20 --warmup 3 > gpurun_out/pn/ab.json 2> gpurun_out/pn/ab.err || { tail -5 gpurun_out/pn/ab.err; exit 4; }
    echo "mixtral DLS_POST_NORM=$v $(python -c 'import json;print(json.load(open("gpurun_out/pn/ab.json"))["ms_per_step"])')"
  done
done
cd /tmp && export TMPDIR=/tmp
DLS_POST_NORM=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pn/prof" -o mixtral -- \
  python3 "$ROOT/bench.py" --model mixtral-8x7b --steps 3 --warmup 2 --no-graph > "$ROOT/gpurun_out/pn/prof.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/pn/prof.log"; exit 5; }
cd "$ROOT" && python tools/analyze_trace.py gpurun_out/pn/prof/mixtral_kernel_trace.csv --steps 2 > gpurun_out/pn/mixtral_breakdown.txt && head -18 gpurun_out/pn/mixtral_breakdown.txt
