set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_batch; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_devp2p.py tests/test_loopback.py -m gpu -k "device or batched" -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" $O/tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
TICKS=2e8 STEPS=20 timeout -k 10 200 python -u benchmarks/devp2p_check.py expert,expert_dp,pipeline_merged 2,4 > $O/chk.log 2>&1; grep -v amdgpu.ids $O/chk.log | cut -c1-400
timeout -k 10 600 python -u benchmarks/loopback_configs.py --configs mixtral_expert --transport device --steps 5 > $O/mixtral.jsonl 2> $O/mixtral.err || { tail -20 $O/mixtral.err; exit 4; }
cut -c1-900 $O/mixtral.jsonl
