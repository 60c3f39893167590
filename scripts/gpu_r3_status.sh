#!/bin/bash
# Round-3 status on one GPU: every BASELINE config (GPT-2 with the capped / strong extras), the
# host-overhead benchmark in its three issue modes, and a Llama-3-8B rocprofv3 breakdown.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/r3s
export DLS_SKIP_BUILD=1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/r3s/gpt2_extras.json 2> gpurun_out/r3s/gpt2_extras.err || { tail -20 gpurun_out/r3s/gpt2_extras.err; exit 3; }
cat gpurun_out/r3s/gpt2_extras.json
DLS_PREFETCH=1 timeout -k 10 300 python benchmarks/bench_host_overhead.py --model gpt2 --regime 0.8 --json gpurun_out/r3s/host_gpt2.json > gpurun_out/r3s/host_gpt2.log 2>&1 || { tail -20 gpurun_out/r3s/host_gpt2.log; exit 4; }
cat gpurun_out/r3s/host_gpt2.json
timeout -k 10 300 python bench.py --model llama3-8b --steps 20 --no-extras > gpurun_out/r3s/llama.json 2> gpurun_out/r3s/llama.err || { tail -20 gpurun_out/r3s/llama.err; exit 5; }
timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 10 --no-extras > gpurun_out/r3s/mixtral.json 2> gpurun_out/r3s/mixtral.err || { tail -20 gpurun_out/r3s/mixtral.err; exit 6; }
python -c "import json;[print(n, json.load(open(f'gpurun_out/r3s/{n}.json'))['ms_per_step']) for n in ('llama','mixtral')]"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/r3s/prof_llama" -o llama -- python3 "$ROOT/bench.py" --model llama3-8b --steps 5 --warmup 2 --no-extras > "$ROOT/gpurun_out/r3s/prof_llama.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3s/prof_llama.log"; exit 7; }
python3 "$ROOT/tools/analyze_trace.py" "$ROOT/gpurun_out/r3s/prof_llama/llama_kernel_trace.csv" --steps 3 > "$ROOT/gpurun_out/r3s/llama_breakdown.txt" 2>&1
head -30 "$ROOT/gpurun_out/r3s/llama_breakdown.txt"
