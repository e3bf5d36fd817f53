set -o pipefail
mkdir -p gpurun_out/micro
timeout -k 10 120 ./scripts/micro/frameio > gpurun_out/micro/frameio.txt 2>&1 || { echo FAIL; cat gpurun_out/micro/frameio.txt; exit 1; }
cat gpurun_out/micro/frameio.txt
timeout -k 10 120 ./scripts/micro/access > gpurun_out/micro/access2.txt 2>&1 || { echo FAIL; exit 1; }
cat gpurun_out/micro/access2.txt
