# Bench lines of library variants (diagnostic builds; no parity check):
# LIBS="default lib/libdpgpu_x.so" CFGS="2 1"
set -o pipefail
mkdir -p gpurun_out/libs
export TMPDIR=/tmp
for lib in ${LIBS:-default}; do
  for c in ${CFGS:-2}; do
    tag=$(basename $lib .so)_c$c
    if [ "$lib" = default ]; then unset DPGPU_LIB; else export DPGPU_LIB=$PWD/dataplane_amd/$lib; fi
    timeout -k 10 300 python bench.py --config $c --no-cpu --no-host > gpurun_out/libs/$tag.json 2> gpurun_out/libs/$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/libs/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/libs/$tag.json'));print('$tag', d['value'], d['roofline']['kernel_ms'])"
  done
done
