set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export DLS_SKIP_BUILD=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/run1_pytest.log 2>&1
echo "pytest exit $?" >> gpurun_out/run1_pytest.log
tail -5 gpurun_out/run1_pytest.log
