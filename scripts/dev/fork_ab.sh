# NAT suites, then the NAT legs at the given fork points, then kernel traces
# of the masquerade and mixed legs at fork 3 (steady replay right after prep).
set -o pipefail
FORKS="${FORKS:-2 3}" bash scripts/gpu_fork.sh || exit 1
mkdir -p gpurun_out/forktr
for K in masq mixed; do
  DPGPU_REPLAY_FORK=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/forktr/p${K}3 -o run -- \
    python bench.py --nat-only --nat-kind $K --steps 4 > gpurun_out/forktr/${K}3.json 2> gpurun_out/forktr/${K}3.err \
    || { echo TRACE_FAIL $K; tail -20 gpurun_out/forktr/${K}3.err; exit 1; }
done
echo TRACE_OK
