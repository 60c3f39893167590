set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_devp2p; mkdir -p $O
for cfg in "SINGLE=1 STEPS=20" "SINGLE=0 STEPS=2" "SINGLE=1 STEPS=20"; do
  env $cfg timeout -k 10 200 python -u benchmarks/devp2p_check.py sequence,capped_eft 4 > $O/chk_$$.log 2>&1; echo "$cfg:"; grep -v amdgpu.ids $O/chk_$$.log | tail -2
done
