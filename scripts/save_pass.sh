# Copy a gpu_pass.sh pass out of gpurun_out/ into profiles/<dir>/:
#   bash scripts/save_pass.sh profiles/r03/head_<sha> [cfg]
set -e
d=$1; c=${2:-2}
mkdir -p $d
cp gpurun_out/bench.json $d/c${c}_bench.json
cp gpurun_out/prof/run_kernel_stats.csv $d/c${c}_kernel_stats.csv
python3 scripts/pmc_summary.py gpurun_out/pmc > $d/c${c}_pmc.json
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log > $d/pytest_gpu.txt || true
cp gpurun_out/smoke.log $d/smoke.txt
