#!/bin/bash
# A/B of the parameter-refill path (in order vs side-stream prefetch) on capped GPT-2 plans.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
for pf in 0 1; do
  for cm in "reference 0.9,0.8" "bytes 0.6,0.5"; do
    set -- $cm
    name=ab_pf${pf}_$1; mkdir -p gpurun_out/$name
    DLS_PREFETCH=$pf timeout -k 10 300 python simulation.py --execute --out gpurun_out/$name --model gpt2 \
      --schedulers ${SCHEDS:-EFT} --steps 30 --regimes $2 --cost-model $1 > gpurun_out/$name.log 2>&1 \
      || { echo "FAILED $name"; tail -20 gpurun_out/$name.log; exit 3; }
    echo "== prefetch=$pf cost=$1"; grep "^\[execute\]" gpurun_out/$name.log
  done
done
