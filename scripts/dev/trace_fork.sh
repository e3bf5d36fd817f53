set -o pipefail
mkdir -p gpurun_out/forktr
export TMPDIR=/tmp
for F in 2 1; do
DPGPU_REPLAY_FORK=$F timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/forktr/p$F -o run -- \
  python bench.py --nat-only --nat-kind mixed --steps 4 > gpurun_out/forktr/m$F.json 2> gpurun_out/forktr/m$F.err || { echo FAIL; tail -20 gpurun_out/forktr/m$F.err; exit 1; }
done
echo OK
