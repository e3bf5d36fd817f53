# Per-stage wave timing (diagnostic build) for the bench configs.
set -o pipefail
mkdir -p gpurun_out/t
export TMPDIR=/tmp
for c in ${CFGS:-1 2 3 4 5}; do
  timeout -k 10 240 python scripts/stage_timing.py --config $c > gpurun_out/t/c$c.json 2> gpurun_out/t/c$c.err || { echo TIMING_FAIL $c; tail -5 gpurun_out/t/c$c.err; exit 1; }
  cat gpurun_out/t/c$c.json
done
