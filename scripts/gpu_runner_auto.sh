#!/bin/bash
# Issue-mode selection (DLS_RUNNER=auto) on capped Llama-3-8B, and the executor GPU tests.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/rauto; mkdir -p $O
export DLS_SKIP_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_rccl_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cap in 15.5 13.8; do
  timeout -k 10 400 python bench.py --model llama3-8b --cap-gb $cap --steps 10 --warmup 3 --no-extras > $O/l_$cap.json 2> $O/l_$cap.err || { tail -20 $O/l_$cap.err; exit 3; }
  echo "cap $cap $(python -c "import json;d=json.load(open('$O/l_$cap.json'));print(d['ms_per_step'], d['issue_mode'], d['refill_gb_per_step'])")"
done
