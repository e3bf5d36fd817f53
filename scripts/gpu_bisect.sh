# Run one GPU test selection against several library builds: LIBS="libdpgpu_head.so ..." SEL="edge"
set -o pipefail
mkdir -p gpurun_out/bis
export TMPDIR=/tmp
for lib in ${LIBS}; do
  DPGPU_LIB=$PWD/dataplane_amd/lib/$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${SEL:-edge}" > gpurun_out/bis/$lib.log 2>&1
  rc=$?
  echo "$lib rc=$rc $(tail -1 gpurun_out/bis/$lib.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
