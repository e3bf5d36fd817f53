# NAT legs (masquerade, mixed, port forwarding) alternating this tree's
# library and libdpgpu_head.so, two rounds, after the NAT suites.
set -o pipefail
mkdir -p gpurun_out/natab
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_nat_scale.py tests/test_gpu_natmix.py tests/test_gpu_masquerade.py \
  tests/test_gpu_portfw.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/natab/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; tail -40 gpurun_out/natab/pytest.log; exit 1; }
echo PYTEST_OK; grep -E "passed|failed" gpurun_out/natab/pytest.log | tail -1
for r in 1 2; do
  for v in base head; do
    lib=dataplane_amd/lib/libdpgpu.so; [ $v != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
    for K in masq mixed pf; do
      DPGPU_LIB=$lib timeout -k 10 300 python bench.py --nat-only --nat-kind $K --steps 4 > gpurun_out/natab/$v$r$K.json 2> gpurun_out/natab/$v$r$K.err \
        || { echo FAIL $v $K; tail -5 gpurun_out/natab/$v$r$K.err; exit 1; }
    done
    python3 -c "
import json
m=json.load(open('gpurun_out/natab/$v${r}masq.json'))['nat_masquerade']; x=json.load(open('gpurun_out/natab/$v${r}mixed.json'))['nat_mixed']['mixed']
p=json.load(open('gpurun_out/natab/$v${r}pf.json'))['nat_portfw']
print('r$r $v masq', [l['launch_ms_median'] for l in m['legs']], m['established']['launch_ms_median'], 'mixed', x['launch_ms_median'], 'pf', [l['launch_ms_median'] for l in p['legs'] if not l['one_lane']])"
  done
done
