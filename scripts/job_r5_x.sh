set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_x; mkdir -p $O
# cross-request expert batches: index kernel + grouped pair numerics, expert_dp loopback (hub and device)
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_loopback.py -m gpu -k "xbatch or expert" -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR" $O/tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
# BASELINE config 5 at full size on one GPU (8 ranks, device transport): batched vs per-node experts
timeout -k 10 600 python -u benchmarks/loopback_configs.py --configs mixtral_expert --transport device --steps 5 > $O/mixtral_xbatch.jsonl 2> $O/mixtral_xbatch.err || { tail -20 $O/mixtral_xbatch.err; exit 4; }
cut -c1-1200 $O/mixtral_xbatch.jsonl
DLS_MOE_XBATCH=0 timeout -k 10 600 python -u benchmarks/loopback_configs.py --configs mixtral_expert --transport device --steps 5 > $O/mixtral_noxbatch.jsonl 2> $O/mixtral_noxbatch.err || { tail -20 $O/mixtral_noxbatch.err; exit 5; }
cut -c1-1200 $O/mixtral_noxbatch.jsonl
