# SQ instruction mix per library build (DPGPU_LIB) on one config: LIBS="default lib/x.so" CFG=2
set -o pipefail
mkdir -p gpurun_out/sql
export TMPDIR=/tmp
for lib in ${LIBS:-default}; do
  tag=$(basename $lib .so)
  if [ "$lib" = default ]; then unset DPGPU_LIB; else export DPGPU_LIB=$PWD/dataplane_amd/$lib; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/sql/$tag -o run -- python bench.py --config ${CFG:-2} --steps 2 --warmup 1 --no-cpu --no-host > gpurun_out/sql/$tag.json 2> gpurun_out/sql/$tag.err || { echo "PMC $tag failed"; exit 1; }
  echo "== $tag"; python scripts/pmc_kernel.py gpurun_out/sql/$tag | python -c "
import sys
d={l.split()[0]:float(l.split()[1]) for l in sys.stdin if l.strip()}
w=d['SQ_WAVES']; print(' '.join(f'{k[8:] if k.startswith(\"SQ_INSTS\") else k}={d[k]/w:.0f}' for k in sorted(d) if k!='SQ_WAVES'))"
done
# FETCH=1: one FETCH_SIZE pass per library as well (KB per dispatch, as read)
if [ -n "$FETCH" ]; then
for lib in ${LIBS:-default}; do
  tag=$(basename $lib .so)_fetch
  if [ "$lib" = default ]; then unset DPGPU_LIB; else export DPGPU_LIB=$PWD/dataplane_amd/$lib; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sql/$tag -o run -- python bench.py --config ${CFG:-2} --steps 2 --warmup 1 --no-cpu --no-host > gpurun_out/sql/$tag.json 2> gpurun_out/sql/$tag.err || { echo "PMC $tag failed"; exit 1; }
  echo "== $tag"; python scripts/pmc_kernel.py gpurun_out/sql/$tag
done
fi
