# Extra PMC passes (instruction cache, wait states, scratch) on the C2 bench.
set -o pipefail
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
CFG=${CFG:-2}
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmcx/counters.txt 2>&1 || true
i=0
for set in ${SETS:-"SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_IFETCH SQ_WAVES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmcx/p$i -o run -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu --no-host > gpurun_out/pmcx/p$i.json 2> gpurun_out/pmcx/p$i.err || { echo "PMC pass $i failed"; tail -3 gpurun_out/pmcx/p$i.err; }
done
echo END
