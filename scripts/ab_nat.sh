# A/B of the NAT legs between the product library and variants
# (VARIANTS="rw4 rw8": lib/libdpgpu_<v>.so), alternating, one run each.
set -o pipefail
mkdir -p gpurun_out/abn
for v in base ${VARIANTS:-rw4 rw8} base; do
  lib=dataplane_amd/lib/libdpgpu.so
  [ "$v" != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
  DPGPU_LIB=$lib timeout -k 10 300 python3 bench.py --nat-only --steps 5 > gpurun_out/abn/$v.json 2> gpurun_out/abn/$v.err || { echo "FAIL $v"; tail -5 gpurun_out/abn/$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abn/$v.json').read().strip().splitlines()[-1]); print('$v', [(l['pf_share'], l['one_lane'], l['launch_ms_median']) for l in d['nat_portfw']['legs']], [l['launch_ms_median'] for l in d['nat_masquerade']['legs']])"
done
