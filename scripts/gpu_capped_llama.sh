#!/bin/bash
# Llama-3-8B under a per-GPU parameter cap (refills every step): the native step runner with the
# copy-stream prefetch, against the Python issue loop (DLS_RUNNER=0), untraced.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/capl; mkdir -p $O
export DLS_SKIP_BUILD=1
for cap in 15.5 13.8; do
  for r in 1 0; do
    DLS_RUNNER=$r timeout -k 10 400 python bench.py --model llama3-8b --cap-gb $cap --steps 10 --warmup 3 --no-extras > $O/l_${cap}_$r.json 2> $O/l_${cap}_$r.err || { tail -20 $O/l_${cap}_$r.err; exit 3; }
    echo "cap $cap runner $r $(python -c "import json;d=json.load(open('$O/l_${cap}_$r.json'));print(d['ms_per_step'], d['refill_gb_per_step'], d['tasks_completed'])")"
  done
done
