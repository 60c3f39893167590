#!/bin/bash
# Executed evaluation sweeps (simulation.py --execute) on one GPU: GPT-2 and GPT-2-medium under
# the reference memory regimes (0.5 GB per parameter) and under real byte costs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
run() {  # run <name> <timeout> args...
  local name=$1 t=$2; shift 2
  mkdir -p "gpurun_out/$name"
  timeout -k 10 "$t" python simulation.py --execute --out "gpurun_out/$name" "$@" > "gpurun_out/$name.log" 2>&1 \
    || { echo "FAILED $name"; tail -20 "gpurun_out/$name.log"; exit 3; }
  grep "^\[execute\]" "gpurun_out/$name.log"
}
run exec_gpt2_ref 400 --model gpt2 --schedulers DFS,Greedy,Critical,MRU_spec,EFT --steps 20 --regimes 1.0,0.9,0.8,0.6
run exec_gpt2_bytes 400 --model gpt2 --schedulers DFS,Critical,MRU_spec,EFT --steps 20 --regimes 0.8,0.6,0.5 --cost-model bytes
run exec_gpt2m_ref 600 --model gpt2-medium --schedulers DFS,Critical,MRU_spec,EFT --steps 10 --regimes 1.0,0.8,0.6
