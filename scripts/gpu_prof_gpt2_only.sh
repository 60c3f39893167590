#!/bin/bash
# GPT-2 bench + rocprofv3 breakdown only.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/pg; mkdir -p $O
export DLS_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-extras --steps 200 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python -c "import json;print(json.load(open('$O/bench.json'))['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o k -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-extras > "$ROOT/$O/prof.log" 2>&1 || { tail -20 "$ROOT/$O/prof.log"; exit 6; }
python3 "$ROOT/tools/analyze_trace.py" "$ROOT/$O/prof/k_kernel_trace.csv" --steps 5 --per-dispatch > "$ROOT/$O/breakdown.txt" 2>&1
head -12 "$ROOT/$O/breakdown.txt"
