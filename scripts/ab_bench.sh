# A/B of library variants on one box: bench.py kernel-only legs per variant,
# alternating, two rounds.  VARIANTS="base sc1" CONFIGS="2 5" bash scripts/ab_bench.sh
set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2; do
  for c in ${CONFIGS:-2}; do
    for v in ${VARIANTS:-base}; do
      lib=dataplane_amd/lib/libdpgpu.so
      [ "$v" != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
      DPGPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-host ${FLOWS:---no-flows} ${EXTRA:-} --steps 20 --warmup 5 \
        > gpurun_out/ab/${v}_c${c}_r${r}.json 2> gpurun_out/ab/${v}_c${c}_r${r}.err || { echo "FAIL $v c$c"; tail -5 gpurun_out/ab/${v}_c${c}_r${r}.err; exit 1; }
      python - "$v" "$c" "$r" <<'PY'
import json, sys
v, c, r = sys.argv[1:]
d = json.loads(open(f"gpurun_out/ab/{v}_c{c}_r{r}.json").read().strip().splitlines()[-1])
ft = d.get("flow_table", {})
fu = ft.get("full_units", {}).get("mpps_median") if isinstance(ft.get("full_units"), dict) else None
nat = {l["pf_share"]: l["launch_ms_median"] for l in d.get("nat_portfw", {}).get("legs", [])}
print(f"r{r} C{c} {v:10s} value {d['value']:8.1f}  kernel {d['roofline']['kernel_ms']:.4f} ms median {d['roofline']['kernel_ms_median']:.4f}  flows {ft.get('mpps_median')} full {fu} nat {nat}")
PY
    done
  done
done
