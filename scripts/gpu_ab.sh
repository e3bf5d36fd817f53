# A/B of library variants on C1/C2/C4 bench lines: LIBS="default lib/libdpgpu_w3.so"
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/ab/pytest.log; exit 1; }
echo PYTEST_OK
for lib in ${LIBS:-default}; do
  for c in ${CFGS:-2 1 4}; do
    tag=$(basename $lib .so)_c$c
    if [ "$lib" = default ]; then unset DPGPU_LIB; else export DPGPU_LIB=$PWD/dataplane_amd/$lib; fi
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu --no-host > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/ab/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', d['value'], d['roofline']['kernel_ms'])"
  done
done
