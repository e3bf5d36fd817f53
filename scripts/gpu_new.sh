# GPU: the newest tests first, then the flows bench leg.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbuf.py tests/test_gpu_flows.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { echo NEW_FAIL; tail -60 gpurun_out/pytest_new.log; exit 1; }
echo NEW_OK
timeout -k 10 400 python bench.py --no-cpu --no-host > gpurun_out/bench_flows.json 2> gpurun_out/bench_flows.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_flows.err; exit 1; }
echo BENCH_OK
