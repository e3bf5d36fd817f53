# NAT composition / mixed-burst / flow-filter classifier GPU tests, the
# affected NAT and ACL suites, then the mixed NAT leg under rocprofv3 (kernel
# stats).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_natcombo.py tests/test_gpu_ff_classify.py tests/test_acl_classify.py \
  tests/test_gpu_natmix.py tests/test_gpu_masquerade.py tests/test_gpu_portfw.py tests/test_gpu_nat_scale.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_natmix.log 2>&1 \
  || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_natmix.log; exit 1; }
echo PYTEST_OK
grep -E "passed|failed" gpurun_out/pytest_natmix.log | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mix -o run -- \
  python bench.py --nat-only --nat-kind mixed --steps 6 > gpurun_out/natmix_leg.json 2> gpurun_out/natmix_leg.err \
  || { echo LEG_FAIL; tail -30 gpurun_out/natmix_leg.err; exit 1; }
echo LEG_OK
python3 -c "
import json; d=json.load(open('gpurun_out/natmix_leg.json'))['nat_mixed']['mixed']
print(d['launch_ms'], d['launch_ms_median'], d['nat_pass'], d['done_histogram'], d['first_burst_nat_pass'])"
timeout -k 10 600 python -u scripts/dev/hip_runtimes_diag.py > gpurun_out/hip_runtimes_diag.txt 2>&1 || { echo DIAG_FAIL; tail -20 gpurun_out/hip_runtimes_diag.txt; exit 1; }
cat gpurun_out/hip_runtimes_diag.txt
