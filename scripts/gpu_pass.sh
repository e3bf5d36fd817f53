# Full GPU pass: parity tests, smoke, default bench (with CPU baseline),
# rocprofv3 kernel statistics of the same bench command, PMC passes for HBM
# traffic.  Stops at the first failing GPU step.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CFG=${CFG:-2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; cat gpurun_out/smoke.log; exit 1; }
echo SMOKE_OK
timeout -k 10 400 python bench.py --config $CFG > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail gpurun_out/bench.err; exit 1; }
echo BENCH_OK
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --config $CFG --no-cpu --no-host > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo PROF_FAIL; exit 1; }
echo PROF_OK
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu --no-host --no-nat --no-flows > gpurun_out/pmc/p$i.json 2> gpurun_out/pmc/p$i.err || { echo "PMC pass $i failed"; exit 1; }
done
echo END
