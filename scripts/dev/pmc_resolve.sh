# PMC of the NAT pass kernels over the port-forwarding legs (one counter set
# per run).
set -o pipefail
mkdir -p gpurun_out/pmcres
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmcres/p$i -o run -- python bench.py --nat-only --nat-kind pf --steps 2 \
    > gpurun_out/pmcres/p$i.json 2> gpurun_out/pmcres/p$i.err || { echo "PMC pass $i failed"; tail -5 gpurun_out/pmcres/p$i.err; exit 1; }
done
echo PMC_OK
