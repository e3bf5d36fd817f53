# A/B of burst-buffer layouts on the bench configs (no CPU leg).
set -o pipefail
mkdir -p gpurun_out/lay
export TMPDIR=/tmp
for c in ${CFGS:-2 1}; do
  for l in dpdk packed; do
    timeout -k 10 300 python bench.py --config $c --layout $l --no-cpu --no-host > gpurun_out/lay/c${c}_$l.json 2> gpurun_out/lay/c${c}_$l.err || { echo BENCH_FAIL $c $l; tail -5 gpurun_out/lay/c${c}_$l.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/lay/c${c}_$l.json'));print('C$c $l', d['value'], d['roofline']['kernel_ms'])"
  done
done
