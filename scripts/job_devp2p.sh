set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_devp2p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_devp2p.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/ipc.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error" $O/ipc.log | tail -20; tail -3 $O/ipc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_loopback.py -m gpu -k "device_transport" -x -v --timeout 240 --timeout-method thread > $O/loop.log 2>&1; rc=$?; grep -E "PASS|FAIL" $O/loop.log | tail -20; tail -3 $O/loop.log; [ $rc -eq 0 ] || exit $rc
