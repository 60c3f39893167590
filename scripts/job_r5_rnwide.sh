#!/bin/bash
# 512-thread split-K reduce-norm rows (DLS_RN_WIDE=1): fp32 numerics, then same-box A/B on Llama-3-8B / Mixtral
set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_rnwide; mkdir -p $O
DLS_RN_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "post_norm" -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 3; }
tail -2 $O/test.log
TAG=r5_rnwide_llama ROUNDS=3 bash scripts/gpu.sh ab DLS_RN_WIDE 0 1 --model llama3-8b || exit 4
TAG=r5_rnwide_mixtral ROUNDS=2 bash scripts/gpu.sh ab DLS_RN_WIDE 0 1 --model mixtral-8x7b || exit 5
