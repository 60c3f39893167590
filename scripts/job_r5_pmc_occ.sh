#!/bin/bash
# Resident waves per CU of the Mixtral expert launches: the table's tiles (44 / 33, one 512-thread
# workgroup per CU) against the two-workgroups-per-CU tiles (46 / 47) and the same 128x128 tile
# at one workgroup per CU (15). One SQ counter pass per pair (benchmarks/pmc_probe.py moe G D).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export DLS_SKIP_BUILD=1
S1="SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"
for pair in "44 33" "46 46" "47 47" "15 15"; do
  w=$(echo "$pair" | tr ' ' '_')
  TAG=pmc_occ_$w bash scripts/gpu.sh pmc "$S1" python3 "$ROOT/benchmarks/pmc_probe.py" moe $pair || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_occ_$w --match gemm_glds > gpurun_out/pmc_occ_${w}_summary.txt 2>&1
  echo "== gate/up, down configs $pair"; cat gpurun_out/pmc_occ_${w}_summary.txt
done
