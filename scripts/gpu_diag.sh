# Diagnostic GPU pass: parity tests, counter list, and memory-pipeline PMC
# passes (TA / TCP / TCC) on the bench kernel for C1 and C2.
set -o pipefail
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/diag/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/diag/pytest_gpu.log; exit 1; }
echo PYTEST_OK
timeout -s KILL 60 rocprofv3 -L > gpurun_out/diag/counters.txt 2>&1 || echo "counter list failed"
for c in 2 1; do
  timeout -k 10 120 python bench.py --config $c --no-cpu --no-host > gpurun_out/diag/c$c.json 2> gpurun_out/diag/c$c.err || { echo BENCH_FAIL $c; exit 1; }
  cat gpurun_out/diag/c$c.json
  i=0
  for set in "TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" "TD_TD_BUSY_sum TD_BUSY_avr" "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d gpurun_out/diag/pmc_c$c/p$i -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-host > gpurun_out/diag/pmc_c$c_p$i.json 2> gpurun_out/diag/pmc_c${c}_p$i.err || echo "PMC pass $c/$i failed"
  done
done
echo END
