# Build libdpgpu.so of a git revision (default HEAD) into dataplane_amd/lib/libdpgpu_<name>.so
# for A/B runs (scripts/ab_bench.sh VARIANTS="base <name>"), with that revision's own Makefile.
set -e
REV=${1:-HEAD}; NAME=${2:-head}
T=$(mktemp -d)
git archive "$REV" dataplane_amd include | tar -x -C "$T"
make -C "$T/dataplane_amd" -j8 lib/libdpgpu.so
cp "$T/dataplane_amd/lib/libdpgpu.so" "dataplane_amd/lib/libdpgpu_$NAME.so"
rm -rf "$T"
