# The flows suites (flow table, NAT) on this tree's library, then the C2 / C5
# A/B with the flow-table leg against libdpgpu_head.so, then the stage timing
# of the flows variant (diagnostic build).
set -o pipefail
mkdir -p gpurun_out/fab
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_flows.py tests/test_gpu_portfw.py tests/test_gpu_masquerade.py \
  tests/test_gpu_natmix.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/fab/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/fab/pytest.log; exit 1; }
echo PYTEST_OK
grep -E "passed|failed" gpurun_out/fab/pytest.log | tail -1
VARIANTS="base head" CONFIGS="2 5" FLOWS=" " EXTRA="--no-nat" bash scripts/ab_bench.sh || exit 1
if [ -n "$TIMING" ]; then
  for F in "" "--flows"; do
    timeout -k 10 300 python scripts/stage_timing.py --config 2 --meta $F --reps 3 || exit 1
  done
fi
