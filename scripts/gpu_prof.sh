# GPU profiling pass: parity tests, bench, kernel trace, PMC counter passes.
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CFG=${CFG:-2}
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
echo PYTEST_OK
timeout -k 10 400 python bench.py --config $CFG --steps 10 --warmup 3 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; exit 1; }
echo BENCH_OK
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu --no-host > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo PROF_FAIL; exit 1; }
echo PROF_OK
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu --no-host > gpurun_out/pmc/p$i.json 2> gpurun_out/pmc/p$i.err || echo "PMC pass $i failed"
done
echo END
