# Same-box A/B: this tree's libdpgpu.so ("base") against lib/libdpgpu_$V.so,
# two alternating rounds: C2 with the flow-table legs, C1 / C3 / C4 / C5 alone.
set -o pipefail
V=${V:?variant name}
mkdir -p gpurun_out/ab_$V
for r in 1 2; do for v in base $V; do
  lib=dataplane_amd/lib/libdpgpu.so; [ $v != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
  DPGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --no-host --no-nat > gpurun_out/ab_$V/$v${r}c2.json 2> gpurun_out/ab_$V/$v${r}c2.err || { echo FAIL $v c2; tail -5 gpurun_out/ab_$V/$v${r}c2.err; exit 1; }
  for c in 1 3 4 5; do
    DPGPU_LIB=$lib timeout -k 10 300 python bench.py --config $c --no-cpu --no-host --no-nat --no-flows > gpurun_out/ab_$V/$v${r}c$c.json 2> gpurun_out/ab_$V/$v${r}c$c.err || { echo FAIL $v c$c; tail -5 gpurun_out/ab_$V/$v${r}c$c.err; exit 1; }
  done
  python3 -c "
import json
d=json.load(open('gpurun_out/ab_$V/$v${r}c2.json')); f=d['flow_table']
o=[json.load(open('gpurun_out/ab_$V/$v${r}c%d.json'%c))['value'] for c in (1,3,4,5)]
print('r$r $v C2', d['value'], 'flows', f['mpps_median'], f['full_units']['mpps_median'], 'C1 C3 C4 C5', o)"
done; done
