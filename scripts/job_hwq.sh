set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_hwq; mkdir -p $O
for q in 4 16; do timeout -k 10 60 python -u benchmarks/hwq_probe.py $q 20 > $O/q$q.log 2>&1; grep -v amdgpu.ids $O/q$q.log | tail -2; done
