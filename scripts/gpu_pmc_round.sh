#!/bin/bash
# PMC passes over one round of a GEMM config (each pass its own rocprofv3 run).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/pmc
export DLS_SKIP_BUILD=1
CFG=${CFG:-34}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$ROOT/gpurun_out/pmc/counters.txt" 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pmc/p$i" -o r -- python3 "$ROOT/benchmarks/probe_gemm_round.py" --cfg $CFG > "$ROOT/gpurun_out/pmc/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$ROOT/gpurun_out/pmc/p$i.log"; }
done
ls -R "$ROOT/gpurun_out/pmc" | head -30
