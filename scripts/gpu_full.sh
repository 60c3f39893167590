#!/bin/bash
# Full GPU round: tests, smoke, kernel microbench, DAG bench (+profile timeline), rocprofv3 stats.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
step kbench
timeout -k 10 500 python benchmarks/bench_kernels.py ${KBENCH_ARGS:-} > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.err || { tail -20 gpurun_out/kbench.err; exit 4; }
cut -c1-400 gpurun_out/kbench.jsonl
step bench
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -20 gpurun_out/bench1.err; exit 5; }
cat gpurun_out/bench1.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-graph --profile > gpurun_out/bench1_profile.json 2> gpurun_out/bench1_profile.err || { tail -20 gpurun_out/bench1_profile.err; exit 6; }
step rocprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o gpt2 -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-graph > "$ROOT/gpurun_out/prof.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/prof.log"; exit 7; }
head -12 "$ROOT/gpurun_out/prof/gpt2_kernel_stats.csv" | cut -c1-200
cp "$ROOT/distributed_llm_scheduler_amd/ops/gemm_tuning.json" "$ROOT/gpurun_out/" 2>/dev/null || true
