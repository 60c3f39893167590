#!/bin/bash
# Same-box A/B of GEMM tuning tables: alternating bench.py runs, one per table per round.
# entry: table[@VAR=VALUE] (one environment switch per entry)
# usage: TABLES="distributed_llm_scheduler_amd/ops/gemm_tuning.json benchmarks/tuning_ab/lm34.json" \
#        BENCH_ARGS="--model gpt2" ROUNDS=3 bash scripts/gpu_ab_tables.sh
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/abt
export DLS_SKIP_BUILD=1
TAG=${TAG:-ab}
for i in $(seq ${ROUNDS:-3}); do
  for e in $TABLES; do
    t=${e%%@*}; ev=""; [ "$e" != "$t" ] && ev=${e#*@}; ev=${ev//,/ }   # entry: table[@VAR=VALUE[,VAR=VALUE]]
    env DLS_GEMM_TUNING="$t" $ev timeout -k 10 ${TMO:-200} python bench.py --no-extras --steps ${STEPS:-200} --warmup ${WARM:-10} ${BENCH_ARGS:-} > gpurun_out/abt/r.json 2> gpurun_out/abt/r.err || { tail -5 gpurun_out/abt/r.err; exit 3; }
    echo "$TAG $(basename $t) $ev $(python -c 'import json;print(json.load(open("gpurun_out/abt/r.json"))["ms_per_step"])')" | tee -a gpurun_out/abt/$TAG.txt
  done
done
