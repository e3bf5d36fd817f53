# Quick GPU pass: parity tests, then the default bench (C2, CPU baseline and
# host-inclusive path included).  Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
