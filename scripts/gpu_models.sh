#!/bin/bash
# GPU round: all GPU tests, smoke, GPT-2 bench, then the BASELINE model configs on 1 GPU.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
run() {  # run <name> <timeout> cmd...  (stdout -> gpurun_out/<name>.out, stderr -> .err)
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"; local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; tail -25 "gpurun_out/$name.err"; tail -5 "gpurun_out/$name.out"; exit $rc; fi
  tail -c 1500 "gpurun_out/$name.out"; echo
}
if [ -z "$SKIP_TESTS" ]; then
  run pytest_gpu 700 python -m pytest tests -x -q -m gpu
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench_gpt2 300 python bench.py --steps 50 --warmup 5 --trace-out gpurun_out/trace_gpt2.json
for spec in ${MODELS:-"llama3-8b" "mixtral-8x7b"}; do
  run "bench_$spec" 900 python bench.py --model "$spec" --steps 10 --warmup 2
done
cp "$ROOT/distributed_llm_scheduler_amd/ops/gemm_tuning.json" "$ROOT/gpurun_out/" 2>/dev/null || true
