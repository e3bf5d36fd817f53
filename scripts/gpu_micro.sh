# Access-shape calibration (scripts/micro/access.hip): timings, then one PMC
# pass with the TCP / TD / TA counters on the same binary.
set -o pipefail
mkdir -p gpurun_out/micro
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/access > gpurun_out/micro/access.txt 2>&1 || { echo MICRO_FAIL; cat gpurun_out/micro/access.txt; exit 1; }
cat gpurun_out/micro/access.txt
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/micro/pmc -o run -- ./scripts/micro/access > gpurun_out/micro/pmc.txt 2>&1 || echo PMC_FAIL
echo END
