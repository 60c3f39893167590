#!/bin/bash
# Executed A/B on one GPU: streamed loads on the copy stream through the DMA engines
# (DLS_REFILL=dma: hipMemcpyAsync, no CUs) vs the host-pull kernel (DLS_REFILL=pull), Llama-3-8B.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
run() {  # run <name> <timeout> <refill> <prefetch> args...
  local name=$1 t=$2 rf=$3 pf=$4; shift 4
  mkdir -p "gpurun_out/$name"
  DLS_REFILL=$rf DLS_PREFETCH=$pf timeout -k 10 "$t" python simulation.py --execute --out "gpurun_out/$name" "$@" \
    > "gpurun_out/$name.log" 2>&1 || { echo "FAILED $name"; tail -20 "gpurun_out/$name.log"; exit 3; }
  grep "^\[execute\]" "gpurun_out/$name.log"
}
run pf_llama_dma 400 dma auto --model llama3-8b --schedulers EFT --steps 10 --regimes 0.9,0.8,0.6 --cost-model bytes
run pf_llama_dma_off 400 dma 0 --model llama3-8b --schedulers EFT --steps 10 --regimes 0.9,0.8 --cost-model bytes
