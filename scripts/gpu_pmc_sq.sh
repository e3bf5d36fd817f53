# SQ instruction-mix counters (one rocprofv3 --pmc pass per config): CFGS="1 2"
set -o pipefail
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
for c in ${CFGS:-1 2}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/sq/c$c -o run -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu --no-host > gpurun_out/sq/c$c.json 2> gpurun_out/sq/c$c.err || { echo "PMC c$c failed"; exit 1; }
  python scripts/pmc_kernel.py gpurun_out/sq/c$c || true
done
