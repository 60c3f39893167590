#!/bin/bash
# Round-4 starting point on one GPU: the driver's bench command and a rocprofv3 breakdown of GPT-2.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; O=gpurun_out/r4_start; mkdir -p $O
export DLS_SKIP_BUILD=1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-extras > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 4; }
  python -c "import json;print(json.load(open('$O/bench_$i.json'))['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_gpt2" -o k -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-extras > "$ROOT/$O/prof_gpt2.log" 2>&1 || { tail -20 "$ROOT/$O/prof_gpt2.log"; exit 7; }
python3 "$ROOT/tools/analyze_trace.py" "$ROOT/$O/prof_gpt2/k_kernel_trace.csv" --steps 5 --per-dispatch > "$ROOT/$O/breakdown_gpt2.txt" 2>&1
head -80 "$ROOT/$O/breakdown_gpt2.txt"
