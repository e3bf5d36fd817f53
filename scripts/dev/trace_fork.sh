# Kernel traces of the masquerade (established) and mixed NAT legs, replay
# forked after the lane's plan (2) and after the resolve (1).
set -o pipefail
mkdir -p gpurun_out/forktr
export TMPDIR=/tmp
for F in 2 1; do
  for K in masq mixed; do
    DPGPU_REPLAY_FORK=$F timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/forktr/p${K}$F -o run -- \
      python bench.py --nat-only --nat-kind $K --steps 4 > gpurun_out/forktr/$K$F.json 2> gpurun_out/forktr/$K$F.err \
      || { echo FAIL $K $F; tail -20 gpurun_out/forktr/$K$F.err; exit 1; }
  done
done
echo OK
