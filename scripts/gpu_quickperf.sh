# Quick perf check: bench C2, C1 (and any in $CFGS) without CPU baseline / host path.
set -o pipefail
mkdir -p gpurun_out/qp
for c in ${CFGS:-2 1}; do
  timeout -k 10 120 python bench.py --config $c --no-cpu --no-host > gpurun_out/qp/c$c.json 2> gpurun_out/qp/c$c.err || { echo BENCH_FAIL $c; tail -5 gpurun_out/qp/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/qp/c$c.json'));print('C$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['done_histogram'])"
done
