set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_b8; mkdir -p $O
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/orig.json
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/refined.json
DLS_GEMM_TUNING=$O/refined.json timeout -k 10 900 python -u benchmarks/refine_dag.py --model gpt2 --batch 8 --reps 10 > $O/refine.json 2> $O/refine.err || { tail -20 $O/refine.err; exit 4; }
python -c "import json;print(json.load(open('$O/refine.json'))['changes'])"
for i in 1 2 3; do
  for t in refined orig; do
    DLS_GEMM_TUNING=$O/$t.json timeout -k 10 300 python bench.py --batch 8 --steps 50 --warmup 5 --no-extras > $O/b_$t.json 2>/dev/null || exit 5
    echo "$t $(python -c "import json;print(json.load(open('$O/b_$t.json'))['ms_per_step'])")"
  done
done
