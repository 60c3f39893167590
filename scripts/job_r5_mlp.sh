set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_mlp; mkdir -p $O
timeout -k 10 120 gpubin/mlp_stamps 200 > $O/mlp_stamps.txt 2>&1 || { cat $O/mlp_stamps.txt; exit 2; }
cat $O/mlp_stamps.txt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -m gpu -k "every_block" -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" $O/tests.log | tail; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in "DLS_MLP_FUSED=0" "DLS_MLP_FUSED=1 DLS_MLP_PREFETCH=0" "DLS_MLP_FUSED=1 DLS_MLP_PREFETCH=1"; do
    env $v timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-extras > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 3; }
    echo "$r $v $(python -c "import json;d=json.load(open('$O/b.json'));print(d['ms_per_step'], d.get('launches_per_rank'))")" | tee -a $O/ab.txt
  done
done
