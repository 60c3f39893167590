set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_devp2p; mkdir -p $O
timeout -k 10 300 python -u benchmarks/devp2p_check.py sequence,capped_eft,pipeline,tensor 4 > $O/chk4.log 2>&1; grep -v amdgpu.ids $O/chk4.log | tail -5
timeout -k 10 900 python -u -m pytest tests/test_loopback.py tests/test_devp2p.py -m gpu -k "device" -v --timeout 150 --timeout-method thread > $O/loop.log 2>&1; rc=$?; grep -E "PASS|FAIL" $O/loop.log | tail -30; tail -3 $O/loop.log; [ $rc -eq 0 ] || exit $rc
