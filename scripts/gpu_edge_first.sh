# The edge corpus GPU test alone first (short limit), then the whole GPU suite and the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "edge_corpus and 11" --timeout 200 --timeout-method thread > gpurun_out/pytest_edge.log 2>&1 || { echo EDGE_FAIL; tail -30 gpurun_out/pytest_edge.log; exit 1; }
echo EDGE_OK
bash scripts/gpu_testab.sh
