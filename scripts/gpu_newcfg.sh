#!/bin/bash
# New GEMM tile configs (36-40): numerics, LM-head microbenchmark, in-DAG refinement (GPT-2, Llama-3-8B).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/newcfg
export DLS_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/newcfg/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/newcfg/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/bench_lmhead.py --cfgs 36,34,13 --json gpurun_out/newcfg/lmhead.json > gpurun_out/newcfg/lmhead.log 2>&1 || { tail -20 gpurun_out/newcfg/lmhead.log; exit 4; }
grep cfg gpurun_out/newcfg/lmhead.log
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json gpurun_out/newcfg/tuning.json
export DLS_GEMM_TUNING=gpurun_out/newcfg/tuning.json
timeout -k 10 300 python benchmarks/refine_dag.py --model gpt2 --keys 512x50257x768 --cfgs 36,37,34,35 > gpurun_out/newcfg/refine_gpt2.json 2> gpurun_out/newcfg/refine_gpt2.err || { tail -20 gpurun_out/newcfg/refine_gpt2.err; exit 5; }
grep -v amdgpu gpurun_out/newcfg/refine_gpt2.err | tail -12
timeout -k 10 600 python benchmarks/refine_dag.py --model llama3-8b --reps 5 --keys 512x28672x4096s,512x6144x4096,512x4096x4096,512x4096x14336 --cfgs 36,37,38,39,40 > gpurun_out/newcfg/refine_llama.json 2> gpurun_out/newcfg/refine_llama.err || { tail -20 gpurun_out/newcfg/refine_llama.err; exit 6; }
grep -v amdgpu gpurun_out/newcfg/refine_llama.err | tail -40
