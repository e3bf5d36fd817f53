# The replay off the allocating lane forked to the side stream: the NAT
# suites GPU == oracle (every fork point), then the masquerade and mixed NAT
# legs with DPGPU_REPLAY_FORK 0 (no fork), 1 (after the resolve), 2 (after the
# lane's plan).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/fork
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_nat_scale.py tests/test_gpu_natmix.py tests/test_gpu_masquerade.py \
  tests/test_gpu_portfw.py tests/test_gpu_natcombo.py tests/test_gpu_flows.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/fork/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/fork/pytest.log; exit 1; }
echo PYTEST_OK
grep -E "passed|failed" gpurun_out/fork/pytest.log | tail -2
for F in ${FORKS:-1 2 0}; do
  for K in masq mixed; do
    DPGPU_REPLAY_FORK=$F timeout -k 10 300 python bench.py --nat-only --nat-kind $K --steps 6 \
      > gpurun_out/fork/leg_${K}_$F.json 2> gpurun_out/fork/leg_${K}_$F.err \
      || { echo LEG_FAIL $K $F; tail -30 gpurun_out/fork/leg_${K}_$F.err; exit 1; }
    python3 - "$K" "$F" <<'PY'
import json, sys
k, f = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/fork/leg_{k}_{f}.json"))
if k == "mixed":
    m = d["nat_mixed"]["mixed"]
    print("mixed fork", f, m["launch_ms"], m["launch_ms_median"], m["done_histogram"], m["nat_pass"])
else:
    m = d["nat_masquerade"]
    for v in m["legs"] + [m["established"]]:
        print("masq fork", f, v.get("pf_share", "established"), v["launch_ms_median"], v.get("launch_ms"),
              v["nat_pass"]["lane_kticks"], v["nat_pass"]["bulk_served_lane_records"], v["nat_pass"]["bulk_blocks"],
              v["nat_pass"]["allocation_steps"])
PY
  done
done
