# Build libdpgpu.so of a git revision (default HEAD) into dataplane_amd/lib/libdpgpu_<name>.so for A/B runs.
set -e
REV=${1:-HEAD}; NAME=${2:-head}
T=$(mktemp -d)
git archive "$REV" dataplane_amd include | tar -x -C "$T"
(cd "$T/dataplane_amd" && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -w -shared -o lib_ref.so csrc/dp_kernel.hip csrc/dp_runtime.cpp csrc/dp_tables.cpp)
cp "$T/dataplane_amd/lib_ref.so" "dataplane_amd/lib/libdpgpu_$NAME.so"
rm -rf "$T"
