#!/bin/bash
# write-through GEMM outputs (4) vs default-policy stores (0) on Llama-3-8B, round-5 tiles
set -o pipefail
export DLS_SKIP_BUILD=1
TAG=r5_knob_actpol_ll ROUNDS=3 bash scripts/gpu.sh ab DLS_ACT_POL 4 0 --model llama3-8b || exit 4
