#!/bin/bash
# A/B of the refill path (host-pull kernel vs hipMemcpyAsync DMA) on capped GPT-2 plans.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
for rf in ${REFILLS:-pull dma}; do
  for cm in "reference 0.9,0.8,0.6" "bytes 0.6,0.5"; do
    set -- $cm
    name=rf_${rf}_$1; mkdir -p gpurun_out/$name
    DLS_REFILL=$rf timeout -k 10 300 python simulation.py --execute --out gpurun_out/$name --model gpt2 \
      --schedulers ${SCHEDS:-MRU_spec,EFT} --steps 30 --regimes $2 --cost-model $1 > gpurun_out/$name.log 2>&1 \
      || { echo "FAILED $name"; tail -20 gpurun_out/$name.log; exit 3; }
    echo "== refill=$rf cost=$1"; grep "^\[execute\]" gpurun_out/$name.log
  done
done
