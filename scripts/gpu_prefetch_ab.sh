#!/bin/bash
# Executed A/B on one GPU: EFT's planned residency with streamed loads issued ahead on a copy
# stream (DLS_PREFETCH=auto, eager) vs in-order refills in a hipGraph (DLS_PREFETCH=0),
# Llama-3-8B under real byte costs. Then the executor GPU tests.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pf_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/pf_tests.log; exit 3; }
tail -2 gpurun_out/pf_tests.log
run() {  # run <name> <timeout> <prefetch> args...
  local name=$1 t=$2 pf=$3; shift 3
  mkdir -p "gpurun_out/$name"
  DLS_PREFETCH=$pf timeout -k 10 "$t" python simulation.py --execute --out "gpurun_out/$name" "$@" \
    > "gpurun_out/$name.log" 2>&1 || { echo "FAILED $name"; tail -20 "gpurun_out/$name.log"; exit 3; }
  grep "^\[execute\]" "gpurun_out/$name.log"
}
run pf_llama_auto 400 auto --model llama3-8b --schedulers EFT --steps 10 --regimes 0.9,0.8,0.6 --cost-model bytes
run pf_llama_off 400 0 --model llama3-8b --schedulers EFT --steps 10 --regimes 0.9,0.8,0.6 --cost-model bytes
