# Occupancy A/B: the same kernel built for 2 / 3 / 4 waves per SIMD.
set -o pipefail
mkdir -p gpurun_out/occ
for c in 2 1; do
  for lib in occ2 dpgpu occ4; do
    L=dataplane_amd/lib/libdpgpu_$lib.so; [ $lib = dpgpu ] && L=dataplane_amd/lib/libdpgpu.so
    DPGPU_LIB=$PWD/$L timeout -k 10 120 python bench.py --config $c --no-cpu --no-host > gpurun_out/occ/c${c}_$lib.json 2> gpurun_out/occ/c${c}_$lib.err || { echo FAIL $c $lib; tail -3 gpurun_out/occ/c${c}_$lib.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/occ/c${c}_$lib.json'));print('C$c $lib', d['value'], d['roofline']['kernel_ms'])"
  done
done
