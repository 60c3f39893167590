#!/bin/bash
# Executed A/B of EFT's steady-state residency lowering on one GPU: the planned keep set
# (DLS_RESIDENCY=auto, default) vs the replayed policy trace (DLS_RESIDENCY=trace), real byte
# costs, Llama-3-8B and GPT-2 under capped memory regimes.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
run() {  # run <name> <timeout> <residency> args...
  local name=$1 t=$2 res=$3; shift 3
  mkdir -p "gpurun_out/$name"
  DLS_RESIDENCY=$res timeout -k 10 "$t" python simulation.py --execute --out "gpurun_out/$name" "$@" \
    > "gpurun_out/$name.log" 2>&1 || { echo "FAILED $name"; tail -20 "gpurun_out/$name.log"; exit 3; }
  grep "^\[execute\]" "gpurun_out/$name.log"
}
run res_llama_auto 500 auto --model llama3-8b --schedulers EFT,MRU_spec --steps 10 --regimes 0.9,0.8,0.6 --cost-model bytes
run res_llama_trace 400 trace --model llama3-8b --schedulers EFT --steps 10 --regimes 0.9,0.8,0.6 --cost-model bytes
run res_gpt2_auto 300 auto --model gpt2 --schedulers EFT --steps 20 --regimes 0.6,0.5 --cost-model bytes
run res_gpt2_trace 300 trace --model gpt2 --schedulers EFT --steps 20 --regimes 0.6,0.5 --cost-model bytes
