set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_cp; mkdir -p $O
DLS_P2P_WAIT=cp STEPS=2 timeout -k 5 90 python -u benchmarks/devp2p_check.py pipeline 2 > $O/chk1.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/chk1.log | cut -c1-600 | tail -20
