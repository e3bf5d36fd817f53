# HBM traffic of dp_pipeline_kernel<false> for every config (roofline.traffic):
# rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE, L2 hit/miss, one pass each, plus the
# kernel statistics of the same bench command.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcall
for c in ${CFGS:-1 2 3 4 5}; do
  d=gpurun_out/pmcall/c$c
  mkdir -p $d
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d/stats -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-host --no-flows --no-nat > $d/bench.json 2> $d/bench.err || { echo "STATS_FAIL C$c"; tail -5 $d/bench.err; exit 1; }
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $d/p$i -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-host --no-flows --no-nat > $d/p$i.json 2> $d/p$i.err || { echo "PMC_FAIL C$c pass $i"; tail -5 $d/p$i.err; exit 1; }
  done
  python3 scripts/pmc_summary.py $d > $d/summary.json || exit 1
  echo "C$c $(python3 -c "import json;d=json.load(open('$d/summary.json'))['derived'];print(d)")"
done
echo PMC_ALL_OK
