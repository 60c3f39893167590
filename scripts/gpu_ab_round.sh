#!/bin/bash
# Same-box A/B of this tree against the round's starting tree (./abtree, built in-tree):
# GPT-2 (headline), Llama-3-8B and Mixtral-8x7B, alternating runs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/abr; mkdir -p $O
export DLS_SKIP_BUILD=1
run() {  # run <tree> <tag> <timeout> args...
  local t=$1 tag=$2 tmo=$3; shift 3
  timeout -k 10 $tmo python "$t/bench.py" --no-extras "$@" > $O/r.json 2> $O/r.err || { tail -5 $O/r.err; exit 3; }
  echo "$tag $t $(python -c "import json;print(json.load(open('$O/r.json'))['ms_per_step'])")" | tee -a $O/ab.txt
}
for i in 1 2 3; do for t in abtree .; do run $t gpt2 200 --steps 200 --warmup 10; done; done
for i in 1 2; do for t in abtree .; do run $t llama 300 --model llama3-8b --steps 20 --warmup 3; done; done
for t in abtree .; do run $t mixtral 400 --model mixtral-8x7b --steps 10 --warmup 2; done
