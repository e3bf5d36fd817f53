# Full GPU parity suite against a library build, then benches: LIB=lib/libdpgpu_w4.so
set -o pipefail
mkdir -p gpurun_out/lt
export TMPDIR=/tmp
export DPGPU_LIB=$PWD/dataplane_amd/$LIB
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/lt/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/lt/pytest.log; exit 1; }
echo PYTEST_OK $LIB
