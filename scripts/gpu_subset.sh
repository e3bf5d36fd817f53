# A subset (or all) of the GPU suite, then bench.py with the
# given arguments.  TESTS="tests/test_gpu_portfw.py" BENCH="--no-cpu" bash scripts/gpu_subset.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_sub.log; exit 1; }
echo PYTEST_OK
tail -3 gpurun_out/pytest_sub.log
if [ -n "${BENCH+x}" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > gpurun_out/bench_sub.json 2> gpurun_out/bench_sub.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_sub.err; exit 1; }
  echo BENCH_OK
  python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_sub.json").read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step")}), json.dumps(d["roofline"]["kernel_ms"]))
print(json.dumps(d.get("host_inclusive")))
print(json.dumps(d.get("flow_table")))
PY
fi
