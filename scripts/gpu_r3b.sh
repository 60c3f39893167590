#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
bash scripts/gpu_moe41.sh || exit 3
bash scripts/gpu_ab_r3a.sh || exit 4
