# Bench lines for every config (no CPU leg) + per-stage timing build.
set -o pipefail
mkdir -p gpurun_out/all gpurun_out/t
export TMPDIR=/tmp
for c in ${CFGS:-1 2 3 4 5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-flows > gpurun_out/all/c$c.json 2> gpurun_out/all/c$c.err || { echo BENCH_FAIL $c; tail -5 gpurun_out/all/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/all/c$c.json'));print('C$c', d['value'], d['roofline']['kernel_ms'], d.get('host_inclusive_mpps'))"
done
for c in ${TCFGS:-2}; do
  timeout -k 10 240 python scripts/stage_timing.py --config $c > gpurun_out/t/c$c.json 2> gpurun_out/t/c$c.err || { echo TIMING_FAIL $c; tail -5 gpurun_out/t/c$c.err; exit 1; }
  cat gpurun_out/t/c$c.json
done
