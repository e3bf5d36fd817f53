# the NAT suites + port-forwarding legs (scripts/dev/pf_ab.sh), then the C2 /
# C5 kernel A/B of this tree's library against libdpgpu_head.so
set -o pipefail
bash scripts/dev/pf_ab.sh || exit 1
VARIANTS="base head" CONFIGS="2 5" EXTRA="--no-nat" bash scripts/ab_bench.sh
