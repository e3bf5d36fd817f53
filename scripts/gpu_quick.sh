# Quick GPU iteration: parity tests, then C1/C2/C3/C4 bench lines (no CPU baseline).
set -o pipefail
mkdir -p gpurun_out/q
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/q/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/q/pytest.log; exit 1; }
echo PYTEST_OK
for c in ${CFGS:-2 1 3 4 5}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu --no-host > gpurun_out/q/c$c.json 2> gpurun_out/q/c$c.err || { echo BENCH_FAIL $c; tail -5 gpurun_out/q/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/q/c$c.json'));print('C$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
