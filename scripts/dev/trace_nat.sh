# Kernel traces of the masquerade (established) and mixed NAT legs at the
# default fork point.
set -o pipefail
mkdir -p gpurun_out/trnat
export TMPDIR=/tmp
for K in masq mixed pf; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trnat/p$K -o run -- \
    python bench.py --nat-only --nat-kind $K --steps 3 > gpurun_out/trnat/$K.json 2> gpurun_out/trnat/$K.err \
    || { echo FAIL $K; tail -20 gpurun_out/trnat/$K.err; exit 1; }
done
echo OK
