# GPU parity tests, then the bench of the given library builds (default: the product build).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
LIBS="${LIBS:-default}" CFGS="${CFGS:-2 1 4 5}" bash scripts/gpu_benchlibs.sh
