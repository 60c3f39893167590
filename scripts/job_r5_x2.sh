set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_x2; mkdir -p $O
TICKS=2e8 STEPS=5 timeout -k 10 150 python -u benchmarks/devp2p_check.py expert,expert_dp 2,4 > $O/chk.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/chk.log | cut -c1-600 | tail -8
