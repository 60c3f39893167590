#!/bin/bash
# Mixtral's per-model output-store default (ops.ACT_POL_MODEL: 0) vs the global write-through (4)
set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_actpol; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-extras --model mixtral-8x7b > $O/d.json 2> $O/d.err || { tail -5 $O/d.err; exit 3; }
  echo "default $(python -c "import json;print(json.load(open('$O/d.json'))['ms_per_step'])")"
  DLS_ACT_POL=4 timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-extras --model mixtral-8x7b > $O/w.json 2> $O/w.err || { tail -5 $O/w.err; exit 4; }
  echo "DLS_ACT_POL=4 $(python -c "import json;print(json.load(open('$O/w.json'))['ms_per_step'])")"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-extras > $O/g.json 2> $O/g.err || { tail -5 $O/g.err; exit 5; }
  echo "gpt2 default $(python -c "import json;print(json.load(open('$O/g.json'))['ms_per_step'])")"
done
