#!/bin/bash
# GPT-2 flagship round: GPU tests, GEMM retune + in-DAG refinement, clean bench, rocprofv3 stats.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$REFINE" ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 --refine-tuning > gpurun_out/refine_gpt2.out 2> gpurun_out/refine_gpt2.err || { tail -20 gpurun_out/refine_gpt2.err; exit 3; }
  grep "refinement" gpurun_out/refine_gpt2.err | cut -c1-1500
  cp distributed_llm_scheduler_amd/ops/gemm_tuning.json gpurun_out/
fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 4; }
cat gpurun_out/bench1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o gpt2 -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-graph > "$ROOT/gpurun_out/prof.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/prof.log"; exit 6; }
python3 "$ROOT/tools/analyze_trace.py" "$ROOT/gpurun_out/prof/gpt2_kernel_trace.csv" --steps 5 | tee "$ROOT/gpurun_out/gpt2_breakdown.txt"
