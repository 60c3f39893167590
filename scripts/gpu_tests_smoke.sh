#!/bin/bash
# GPU test suite + smoke + the default bench line on the current build.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/ts; mkdir -p $O
export DLS_SKIP_BUILD=1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['issue_mode'], {k: (v.get('tasks_completed'), v.get('ms_per_step')) for k, v in d['capped'].items() if isinstance(v, dict)}, d['strong'].get('ms_per_step'))"
