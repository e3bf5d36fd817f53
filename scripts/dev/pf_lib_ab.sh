# Port-forwarding suites on this tree's library, then the port-forwarding
# legs alternating this library and libdpgpu_head.so (two rounds).
set -o pipefail
mkdir -p gpurun_out/pfab
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfw.py tests/test_gpu_nat_scale.py tests/test_gpu_natmix.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pfab/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; tail -40 gpurun_out/pfab/pytest.log; exit 1; }
echo PYTEST_OK; grep -E "passed|failed" gpurun_out/pfab/pytest.log | tail -1
for r in 1 2; do
  for v in base head; do
    lib=dataplane_amd/lib/libdpgpu.so; [ $v != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
    DPGPU_LIB=$lib timeout -k 10 300 python bench.py --nat-only --nat-kind pf --steps 4 > gpurun_out/pfab/$v$r.json 2> gpurun_out/pfab/$v$r.err \
      || { echo FAIL $v; tail -5 gpurun_out/pfab/$v$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/pfab/$v$r.json'))['nat_portfw']
print('r$r $v', [(l['pf_share'], l['launch_ms_median']) for l in d['legs'] if not l['one_lane']])"
  done
done
