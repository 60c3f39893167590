#!/bin/bash
# layer weights DMA'd nt above a size (DLS_WEIGHT_NT_MB) on this round's tiles: Mixtral's attention
# weights (>= 20 MB), Llama-3-8B's MLP weights only (>= 100 MB: gate/up 235 MB, down 117 MB)
set -o pipefail
export DLS_SKIP_BUILD=1
TAG=r5_knob_wnt_mx ROUNDS=2 bash scripts/gpu.sh ab DLS_WEIGHT_NT_MB 0 20 --model mixtral-8x7b || exit 4
TAG=r5_knob_wnt_ll ROUNDS=2 bash scripts/gpu.sh ab DLS_WEIGHT_NT_MB 0 100 --model llama3-8b || exit 5
