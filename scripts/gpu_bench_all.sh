#!/bin/bash
# One-GPU bench of every BASELINE config this box can run (JSON lines into gpurun_out/bench_all/).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/bench_all
export DLS_SKIP_BUILD=1
b() {  # b <name> <timeout> args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "gpurun_out/bench_all/$name.json" 2> "gpurun_out/bench_all/$name.err" \
    || { echo "FAILED $name"; tail -20 "gpurun_out/bench_all/$name.err"; exit 3; }
  echo "$name $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['tasks_completed'], d['tasks_total'], d.get('refill_gb_per_step'))" "gpurun_out/bench_all/$name.json")"
}
b gpt2 200
b llama3-8b 300 --model llama3-8b --steps 20
b mixtral-8x7b 400 --model mixtral-8x7b --steps 10
b gpt2m_cap8_mru 300 --model gpt2-medium --cap-gb 8 --cost-model reference --scheduler MRU_spec --steps 20
b gpt2m_cap8_eft 300 --model gpt2-medium --cap-gb 8 --cost-model reference --scheduler EFT --steps 20
