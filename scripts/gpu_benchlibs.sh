# Bench several library builds (no tests), interleaved over REPS rounds:
#   LIBS="default lib/libdpgpu_head.so" CFGS="2 1 4" REPS=2 [FLOWS=1: also the flow-table leg]
set -o pipefail
mkdir -p gpurun_out/bl
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-1}); do
for c in ${CFGS:-2 1 4}; do
  for lib in ${LIBS:-default}; do
    tag=$(basename $lib .so)_c${c}_r$rep
    if [ "$lib" = default ]; then unset DPGPU_LIB; else export DPGPU_LIB=$PWD/dataplane_amd/$lib; fi
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu --no-host $( [ -z "$FLOWS" ] && echo --no-flows ) > gpurun_out/bl/$tag.json 2> gpurun_out/bl/$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/bl/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bl/$tag.json'));print('$tag', d['value'], d['roofline']['kernel_ms'], d.get('flow_table', {}).get('mpps_median', ''))"
  done
done
done
