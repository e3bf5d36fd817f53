# Parity tests, then bench ablations (each a separate process).
set -o pipefail
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
run() { name=$1; shift; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-host "$@" > gpurun_out/abl/$name.json 2> gpurun_out/abl/$name.err || { echo "FAIL $name"; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('gpurun_out/abl/$name.json'));print(d['value'], d['roofline']['kernel_ms'])")"; }
run c2 --config 2
run c2_acl1 --config 2 --acl 1
run c2_acl1_nat1 --config 2 --acl 1 --nat 1
run c1_1m --config 1 --routes-v4 1000000
run c1 --config 1
run c3 --config 3
run c4 --config 4
run c5 --config 5
echo END
