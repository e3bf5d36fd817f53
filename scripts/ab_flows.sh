# A/B of the flows bench leg between the product library and a variant
# (VARIANT=late: lib/libdpgpu_late.so), alternating, two runs each.
set -o pipefail
mkdir -p gpurun_out/abf
for r in 1 2; do
  for v in base ${VARIANT:-late}; do
    lib=dataplane_amd/lib/libdpgpu.so
    [ "$v" != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
    DPGPU_LIB=$lib timeout -k 10 300 python3 bench.py --no-nat --no-cpu --no-host --steps 20 > gpurun_out/abf/$v$r.json 2> gpurun_out/abf/$v$r.err || { echo "FAIL $v $r"; tail -5 gpurun_out/abf/$v$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abf/$v$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['flow_table']['mpps_median'], d['flow_table']['launch_ms_median'])"
  done
done
