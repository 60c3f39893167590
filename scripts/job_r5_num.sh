set -o pipefail
export DLS_SKIP_BUILD=1
O=gpurun_out/r5_num; mkdir -p $O
timeout -k 10 400 python -u benchmarks/gpt2_layer_errors.py > $O/layers.txt 2>&1; rc=$?; cat $O/layers.txt | grep -v amdgpu.ids; exit $rc
