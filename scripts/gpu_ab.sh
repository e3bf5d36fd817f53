# Library A/B: bench each config in $CFGS with each library in $LIBS
# (names under dataplane_amd/lib, "dpgpu" = the product build).
set -o pipefail
mkdir -p gpurun_out/ab
for c in ${CFGS:-2 1}; do
  for lib in ${LIBS:-dpgpu}; do
    L=dataplane_amd/lib/lib$lib.so
    DPGPU_LIB=$PWD/$L timeout -k 10 120 python bench.py --config $c --no-cpu --no-host > gpurun_out/ab/c${c}_$lib.json 2> gpurun_out/ab/c${c}_$lib.err || { echo FAIL $c $lib; tail -3 gpurun_out/ab/c${c}_$lib.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab/c${c}_$lib.json'));print('C$c $lib', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
