# Round-6 full pass: scripts/gpu_pass.sh (every GPU test, smoke, the default
# bench line with all legs, rocprofv3 stats, PMC), then the HIP runtime
# diagnostic (scripts/dev/hip_runtimes_diag.py, 144 classify calls per leg).
set -o pipefail
bash scripts/gpu_pass.sh || exit 1
timeout -k 10 900 python -u scripts/dev/hip_runtimes_diag.py > gpurun_out/hip_runtimes_diag.txt 2>&1 || { echo DIAG_FAIL; tail -20 gpurun_out/hip_runtimes_diag.txt; exit 1; }
cat gpurun_out/hip_runtimes_diag.txt
