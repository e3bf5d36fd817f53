# Instruction-fetch counters of dp_pipeline_kernel<false> on one config (CFG, default 2)
set -o pipefail
mkdir -p gpurun_out/ic
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_WAVES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d gpurun_out/ic/p$i -o run -- python bench.py --config ${CFG:-2} --steps 2 --warmup 1 --no-cpu --no-host --no-flows > gpurun_out/ic/p$i.json 2> gpurun_out/ic/p$i.err || { echo "pass $i failed"; tail -5 gpurun_out/ic/p$i.err; exit 1; }
  python scripts/pmc_kernel.py gpurun_out/ic/p$i
done
