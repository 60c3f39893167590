#!/bin/bash
# write-through GEMM outputs (DLS_ACT_POL=4, measured on GPT-2 / Llama in round 4) on Mixtral
set -o pipefail
export DLS_SKIP_BUILD=1
TAG=r5_knob_actpol_mx ROUNDS=2 bash scripts/gpu.sh ab DLS_ACT_POL 4 0 --model mixtral-8x7b || exit 4
