#!/bin/bash
# One GPU round: kernel/executor tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 4; }
cat gpurun_out/bench1.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-graph --profile > gpurun_out/bench1_profile.json 2> gpurun_out/bench1_profile.err || { tail -20 gpurun_out/bench1_profile.err; exit 5; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o gpt2 -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-graph > "$ROOT/gpurun_out/prof.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/prof.log"; exit 6; }
ls -R "$ROOT/gpurun_out/prof" | head -20
