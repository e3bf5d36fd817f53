# Whole GPU suite, then C2 / C3 / C5 / C1 bench.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/bin
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK; tail -1 gpurun_out/pytest_gpu.log
for c in ${CFGS:-2 3 5 1}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-host --no-flows > gpurun_out/bin/c$c.json 2> gpurun_out/bin/c$c.err || { echo BENCH_FAIL $c; tail -5 gpurun_out/bin/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bin/c$c.json'));print('C$c', d['value'], d['roofline']['kernel_ms'])"
done
