# Bench several library builds (no tests): LIBS="lib/a.so lib/b.so" CFGS="2 1 4"
set -o pipefail
mkdir -p gpurun_out/bl
export TMPDIR=/tmp
for lib in ${LIBS}; do
  for c in ${CFGS:-2 1 4}; do
    tag=$(basename $lib .so)_c$c
    if [ "$lib" = default ]; then unset DPGPU_LIB; else export DPGPU_LIB=$PWD/dataplane_amd/$lib; fi
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu --no-host > gpurun_out/bl/$tag.json 2> gpurun_out/bl/$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/bl/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bl/$tag.json'));print('$tag', d['value'], d['roofline']['kernel_ms'])"
  done
done
