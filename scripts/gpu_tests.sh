# A subset of the GPU suite: TESTS="tests/test_gpu_portfw.py tests/test_gpu_flows.py"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_sub.log; exit 1; }
echo PYTEST_OK
tail -3 gpurun_out/pytest_sub.log
