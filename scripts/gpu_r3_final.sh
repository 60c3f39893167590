#!/bin/bash
# Round-3 final check on one GPU: full GPU test suite, smoke, the driver's bench command (with the
# capped / strong sub-results), every BASELINE model, rocprofv3 kernel stats of GPT-2 and Llama-3-8B.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; O=gpurun_out/r3f; mkdir -p $O
export DLS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 100 --warmup 10 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || { tail -20 $O/bench_gpt2.err; exit 4; }
cut -c1-400 $O/bench_gpt2.json
timeout -k 10 300 python bench.py --model llama3-8b --steps 20 --no-extras > $O/bench_llama.json 2> $O/bench_llama.err || { tail -20 $O/bench_llama.err; exit 5; }
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 10 --no-extras > $O/bench_mixtral.json 2> $O/bench_mixtral.err || { tail -20 $O/bench_mixtral.err; exit 6; }
python -c "import json;[print(n, json.load(open(f'$O/bench_{n}.json'))['ms_per_step']) for n in ('gpt2','llama','mixtral')]"
cd /tmp && export TMPDIR=/tmp
for m in gpt2 llama3-8b; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_$m" -o k -- python3 "$ROOT/bench.py" --model $m --steps 10 --warmup 3 --no-extras > "$ROOT/$O/prof_$m.log" 2>&1 || { tail -20 "$ROOT/$O/prof_$m.log"; exit 7; }
  python3 "$ROOT/tools/analyze_trace.py" "$ROOT/$O/prof_$m/k_kernel_trace.csv" --steps 5 --per-dispatch > "$ROOT/$O/breakdown_$m.txt" 2>&1
  head -14 "$ROOT/$O/breakdown_$m.txt"
done
