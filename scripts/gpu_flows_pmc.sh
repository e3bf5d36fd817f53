# PMC of the flows leg's first-pass kernel (the lean meta unit,
# dp_pipeline_kernel<true, true, false, 6>): FETCH_SIZE, WRITE_SIZE, L2 hit /
# miss and the instruction mix, one pass each, plus kernel statistics.
set -o pipefail
export TMPDIR=/tmp
d=gpurun_out/flowspmc
mkdir -p $d
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d/stats -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-host --no-nat > $d/bench.json 2> $d/bench.err || { echo STATS_FAIL; exit 1; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $d/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-host --no-nat > $d/p$i.json 2> $d/p$i.err || { echo "PMC_FAIL pass $i"; exit 1; }
done
echo FLOWS_PMC_OK
