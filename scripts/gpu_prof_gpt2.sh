#!/bin/bash
# GPT-2 bench + per-dispatch rocprofv3 breakdown (no test suite).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
OUT=${OUT:-gpurun_out/prof_gpt2}
mkdir -p "$ROOT/$OUT"
timeout -k 10 300 python bench.py --steps 100 --warmup 10 ${BENCH_ARGS} > $OUT/bench1.json 2> $OUT/bench1.err || { tail -20 $OUT/bench1.err; exit 4; }
cat $OUT/bench1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o gpt2 -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 ${BENCH_ARGS} > "$ROOT/$OUT/prof.log" 2>&1 || { tail -20 "$ROOT/$OUT/prof.log"; exit 6; }
python3 "$ROOT/tools/analyze_trace.py" "$ROOT/$OUT/prof/gpt2_kernel_trace.csv" --steps 5 --per-dispatch > "$ROOT/$OUT/breakdown.txt" 2>&1 || python3 "$ROOT/tools/analyze_trace.py" "$ROOT/$OUT/prof/gpt2_kernel_trace.csv" --steps 5 > "$ROOT/$OUT/breakdown.txt"
cat "$ROOT/$OUT/breakdown.txt" | head -30
