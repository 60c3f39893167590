set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r6lm; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_gemm_shapes and (48 or 49)" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/t.json
DLS_GEMM_TUNING=$O/t.json timeout -k 10 400 python benchmarks/refine_dag.py --model gpt2 --cfgs 48,49 --keys 512x50257x768 > $O/refine_gpt2.log 2>&1 || { tail -20 $O/refine_gpt2.log; exit 4; }
tail -5 $O/refine_gpt2.log
