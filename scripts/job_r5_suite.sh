set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_suite; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
cut -c1-400 $O/bench.json
