#!/bin/bash
# Hardware counters of the LM head and the Mixtral grouped expert launches (benchmarks/pmc_probe.py):
# one rocprofv3 --pmc pass per counter set (within the per-block limits), each under its own limit.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export DLS_SKIP_BUILD=1
S1="SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"
S2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"
S3="SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY SQ_LEVEL_WAVES"
# probes: arguments of benchmarks/pmc_probe.py, one quoted string each (default: lmhead moe)
[ $# -gt 0 ] || set -- lmhead moe
for probe in "$@"; do
  w=$(echo "$probe" | tr ' ' '_')
  i=0
  for set in "$S1" "$S2" "$S3"; do
    i=$((i+1))
    TAG=pmc_${w}_$i bash scripts/gpu.sh pmc "$set" python3 "$ROOT/benchmarks/pmc_probe.py" $probe || exit $?
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${w}_* > gpurun_out/pmc_${w}_summary.txt 2>&1
  cat gpurun_out/pmc_${w}_summary.txt
done
