# Every NAT / flow-table GPU suite, then the port-forwarding, masquerade and
# mixed legs.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/nat
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfw.py tests/test_gpu_nat_scale.py tests/test_gpu_natmix.py \
  tests/test_gpu_masquerade.py tests/test_gpu_natcombo.py tests/test_gpu_flows.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/nat/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/nat/pytest.log; exit 1; }
echo PYTEST_OK
grep -E "passed|failed" gpurun_out/nat/pytest.log | tail -1
for K in pf masq mixed; do
  timeout -k 10 300 python bench.py --nat-only --nat-kind $K --steps 6 > gpurun_out/nat/leg_$K.json 2> gpurun_out/nat/leg_$K.err \
    || { echo LEG_FAIL $K; tail -20 gpurun_out/nat/leg_$K.err; exit 1; }
done
python3 -c "
import json
p=json.load(open('gpurun_out/nat/leg_pf.json'))['nat_portfw']
m=json.load(open('gpurun_out/nat/leg_masq.json'))['nat_masquerade']; x=json.load(open('gpurun_out/nat/leg_mixed.json'))['nat_mixed']['mixed']
print('pf', [(l['pf_share'], l['launch_ms_median'], l['one_lane'], l['prefilled_flows'] > 0) for l in p['legs']])
print('masq', [l['launch_ms_median'] for l in m['legs']], m['established']['launch_ms_median'], m['established']['launch_ms'])
print('mixed', x['launch_ms_median'], x['launch_ms'])"
