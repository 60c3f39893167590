#!/bin/bash
# Configs 42/43 (64x48 tiles, split-K with the in-launch combine) on GPT-2's N = 768 GEMMs:
# tests, then in-DAG timing against the current choices (fc2 K = 3072, out-proj K = 768).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; O=gpurun_out/n768; mkdir -p $O
export DLS_SKIP_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm_shapes or splitk_epilogue or row_stats or folded_norm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/tuning.json
export DLS_GEMM_TUNING=$O/tuning.json
timeout -k 10 400 python benchmarks/refine_dag.py --model gpt2 --reps 30 --keys 512x768x3072,512x768x768 --cfgs 42,43,27 > $O/refine.json 2> $O/refine.err || { tail -20 $O/refine.err; exit 5; }
grep -v amdgpu $O/refine.err | tail -20
