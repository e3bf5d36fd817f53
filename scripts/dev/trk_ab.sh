set -o pipefail
mkdir -p gpurun_out/trk
for r in 1 2; do for v in base trk; do
  lib=dataplane_amd/lib/libdpgpu.so; [ $v != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
  DPGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-host --no-nat > gpurun_out/trk/$v$r.json 2> gpurun_out/trk/$v$r.err || { echo FAIL $v; tail -5 gpurun_out/trk/$v$r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/trk/$v$r.json')); f=d['flow_table']
print('r$r $v', d['value'], d['mpps_median_step'], f['mpps_median'], f['full_units']['mpps_median'])"
done; done
