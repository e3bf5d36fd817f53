# C5 check: full-size parity for C5 and C2, then C5 / C2 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "full_size" > gpurun_out/pytest_fs.log 2>&1 || { echo FS_FAIL; tail -40 gpurun_out/pytest_fs.log; exit 1; }
echo FS_OK
for c in 5 2; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-host --no-flows > gpurun_out/c$c.json 2> gpurun_out/c$c.err || { echo BENCH_FAIL $c; tail -5 gpurun_out/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c$c.json'));print('C$c', d['value'], d['roofline']['kernel_ms'])"
done
