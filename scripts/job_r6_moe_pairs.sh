# Mixtral-8x7B grouped expert launches re-refined in the step's hipGraph with the partner blocks on
# (DLS_EXPERT_PAIRS=2, the default): a heavy expert's second row tile no longer doubles its blocks'
# time, so smaller row tiles may pay now
set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r6moe_pairs; mkdir -p $O
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/t.json
DLS_GEMM_TUNING=$O/t.json timeout -k 10 900 python -u benchmarks/refine_dag.py --model mixtral-8x7b \
  --cfgs 28,29,30,31,32,33,41,44,46,47,14,43 --keys 128x4096x14336g,128x28672x4096sg --min-gain 0.005 \
  > $O/refine.log 2>&1 || { tail -20 $O/refine.log; exit 4; }
grep -v amdgpu $O/refine.log | tail -40
