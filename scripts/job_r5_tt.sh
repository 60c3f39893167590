set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_tt; mkdir -p $O
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/gemm_tuning.json
timeout -k 10 400 python -u -m pytest tests/test_loopback.py -m gpu -k "capped_eft or pipeline_merged" -x -v --timeout 240 --timeout-method thread > $O/loopback.log 2>&1 || { tail -30 $O/loopback.log; exit 5; }
tail -3 $O/loopback.log
timeout -k 10 400 python benchmarks/measure_task_times.py --models gpt2 gpt2-medium llama3-8b --out $O/task_times.json > $O/tt.log 2>&1 || { tail -30 $O/tt.log; exit 6; }
tail -4 $O/tt.log
DLS_GEMM_TUNING=$PWD/$O/gemm_tuning.json timeout -k 10 600 python bench.py --steps 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 7; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], json.dumps(d.get('strong')), json.dumps(d.get('capped'))[:800])"
