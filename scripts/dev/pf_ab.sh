# NAT suites, then the port-forwarding legs (the table emptied between
# launches: every connection created anew) and the mixed leg.
set -o pipefail
mkdir -p gpurun_out/pf
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfw.py tests/test_gpu_nat_scale.py tests/test_gpu_natmix.py \
  tests/test_gpu_masquerade.py tests/test_gpu_natcombo.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pf/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pf/pytest.log; exit 1; }
echo PYTEST_OK
grep -E "passed|failed" gpurun_out/pf/pytest.log | tail -1
timeout -k 10 300 python bench.py --nat-only --nat-kind pf --steps 6 > gpurun_out/pf/leg_pf.json 2> gpurun_out/pf/leg_pf.err \
  || { echo LEG_FAIL; tail -20 gpurun_out/pf/leg_pf.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/pf/leg_pf.json'))['nat_portfw']
print([(l['pf_share'], l['launch_ms_median'], l['one_lane'], l['prefilled_flows']) for l in d['legs']])"
