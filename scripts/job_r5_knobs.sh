#!/bin/bash
# re-check two round-4 knobs on this round's tiles: expert weights nt vs default policy (Mixtral),
# XCD-blocked tile order for plain GEMMs (Llama-3-8B; measured on GPT-2 only before)
set -o pipefail
export DLS_SKIP_BUILD=1
TAG=r5_knob_nt ROUNDS=2 bash scripts/gpu.sh ab DLS_EXPERT_NT 1 0 --model mixtral-8x7b || exit 4
TAG=r5_knob_xcd ROUNDS=2 bash scripts/gpu.sh ab DLS_XCD_BLOCK 0 1 --model llama3-8b || exit 5
