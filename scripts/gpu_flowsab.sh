# Flow-table tests with the default build, then the bench's flow-table leg per library (LIBS), REPS rounds
set -o pipefail
mkdir -p gpurun_out/fab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_flows.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fab/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/fab/pytest.log; exit 1; }
tail -1 gpurun_out/fab/pytest.log
for rep in $(seq 1 ${REPS:-2}); do
  for lib in ${LIBS:-default}; do
    tag=$(basename $lib .so)_r$rep
    if [ "$lib" = default ]; then unset DPGPU_LIB; else export DPGPU_LIB=$PWD/dataplane_amd/$lib; fi
    timeout -k 10 300 python bench.py --config ${CFG:-2} --no-cpu --no-host > gpurun_out/fab/$tag.json 2> gpurun_out/fab/$tag.err || { echo BENCH_FAIL $tag; tail -5 gpurun_out/fab/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/fab/$tag.json'));print('$tag', d['value'], d['flow_table']['mpps_median'], d['flow_table']['launch_ms_median'])"
  done
done
