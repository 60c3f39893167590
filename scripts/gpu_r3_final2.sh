#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
bash scripts/gpu_r3_final.sh || exit 3
bash scripts/gpu_capped_llama.sh || exit 4
