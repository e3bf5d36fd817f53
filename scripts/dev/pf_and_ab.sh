# the NAT suites + port-forwarding legs (scripts/dev/pf_ab.sh), the
# masquerade and mixed legs, then the C2 / C5 kernel A/B of this tree's
# library against libdpgpu_head.so
set -o pipefail
bash scripts/dev/pf_ab.sh || exit 1
for K in masq mixed; do
  timeout -k 10 300 python bench.py --nat-only --nat-kind $K --steps 6 > gpurun_out/pf/leg_$K.json 2> gpurun_out/pf/leg_$K.err \
    || { echo LEG_FAIL $K; tail -20 gpurun_out/pf/leg_$K.err; exit 1; }
done
python3 -c "
import json
m=json.load(open('gpurun_out/pf/leg_masq.json'))['nat_masquerade']; x=json.load(open('gpurun_out/pf/leg_mixed.json'))['nat_mixed']['mixed']
print('masq', [l['launch_ms_median'] for l in m['legs']], m['established']['launch_ms_median'], m['established']['launch_ms'])
print('mixed', x['launch_ms_median'], x['launch_ms'])"
VARIANTS="base head" CONFIGS="2 5" EXTRA="--no-nat" bash scripts/ab_bench.sh
