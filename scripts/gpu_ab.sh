# A/B bench of library builds, no tests: LIBS="default lib/x.so" CFGS="2 1"
set -o pipefail
LIBS="${LIBS:-default}" CFGS="${CFGS:-2 1}" bash scripts/gpu_benchlibs.sh
