# GPU: flow-table tests first (new code), then the whole GPU suite.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_flows.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_flows.log 2>&1 || { echo FLOWS_FAIL; tail -60 gpurun_out/pytest_flows.log; exit 1; }
echo FLOWS_OK
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
tail -3 gpurun_out/pytest_gpu.log
