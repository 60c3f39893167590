#!/bin/bash
# Time one round of GEMM configs hot / cold, then L2 hit-rate counters of the cold run.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/probe
export DLS_SKIP_BUILD=1
for c in 34 8 10; do
  bm=256; bn=256; [ $c = 10 ] && bn=128
  for mode in "--hot" "" "--rotate 4"; do
    timeout -k 10 60 python3 benchmarks/probe_gemm_round.py --cfg $c --bn $bn --reps 20 $mode 2>&1 | grep cfg || exit 3
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d "$ROOT/gpurun_out/probe/tcc" -o r -- python3 "$ROOT/benchmarks/probe_gemm_round.py" --cfg 34 --rotate 4 > "$ROOT/gpurun_out/probe/tcc.log" 2>&1 || { echo "tcc pass failed"; tail -5 "$ROOT/gpurun_out/probe/tcc.log"; }
