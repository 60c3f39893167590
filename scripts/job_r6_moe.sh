# Mixtral-8x7B grouped expert launches: 256-row tiles (one pass up to 256 routed rows) against
# the table's 192-row (down) / 160-row (gate/up) tiles, timed inside the real step's hipGraph
set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r6moe; mkdir -p $O
cp distributed_llm_scheduler_amd/ops/gemm_tuning.json $O/t.json
DLS_GEMM_TUNING=$O/t.json timeout -k 10 700 python -u benchmarks/refine_dag.py --model mixtral-8x7b --cfgs 14,43,0,10,12,29,41 \
  --keys 128x4096x14336g,128x28672x4096sg --min-gain 0.005 > $O/refine.log 2>&1 || { tail -20 $O/refine.log; exit 4; }
grep -v amdgpu $O/refine.log | tail -30
