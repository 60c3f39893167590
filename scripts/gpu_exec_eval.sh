#!/bin/bash
# Executed evaluation sweeps (simulation.py --execute) on one GPU: GPT-2 under the reference
# memory regimes with the in-order and the prefetched refill paths, and the bytes cost model.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
run() {  # run <name> <timeout> args...
  local name=$1 t=$2; shift 2
  mkdir -p "gpurun_out/$name"
  timeout -k 10 "$t" python simulation.py --execute --out "gpurun_out/$name" "$@" > "gpurun_out/$name.log" 2>&1 \
    || { echo "FAILED $name"; tail -20 "gpurun_out/$name.log"; exit 3; }
  grep -A40 "=== EXECUTED" "gpurun_out/$name.log"
}
run exec_gpt2_ref 400 --model gpt2 --schedulers ${SCHEDS:-DFS,Critical,MRU_spec,EFT} --steps 20 --regimes 1.0,0.9,0.8,0.6
DLS_PREFETCH=1 run exec_gpt2_ref_prefetch 400 --model gpt2 --schedulers MRU_spec,EFT --steps 20 --regimes 0.9,0.8,0.6
run exec_gpt2_bytes 400 --model gpt2 --schedulers MRU_spec,EFT --steps 20 --regimes 0.8,0.6,0.5 --cost-model bytes
DLS_PREFETCH=1 run exec_gpt2_bytes_prefetch 400 --model gpt2 --schedulers MRU_spec,EFT --steps 20 --regimes 0.8,0.6,0.5 --cost-model bytes
