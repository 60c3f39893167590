set -o pipefail
export DLS_SKIP_BUILD=1
for m in gpt2 llama3-8b mixtral-8x7b; do
  TAG=r5_final timeout -k 10 500 bash scripts/gpu.sh prof $m > /dev/null || exit 5
  head -12 gpurun_out/r5_final/breakdown_$m.txt
done
for m in llama3-8b mixtral-8x7b; do
  timeout -k 10 400 python bench.py --model $m --steps 30 --warmup 5 --no-extras > gpurun_out/r5_final/bench_$m.json 2> gpurun_out/r5_final/bench_$m.err || { tail -5 gpurun_out/r5_final/bench_$m.err; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/r5_final/bench_$m.json'));print('$m', d['ms_per_step'], d['launches_per_rank'])"
done
