# Which stage's table lines cost the HBM traffic: FETCH_SIZE and the L2
# hit / miss counters of dp_pipeline_kernel<false, false> per config, for the
# product library and for builds with one stage compiled out
# (DP_PROBE_NOACL / NONAT / NOIPF2: `make variant`; their outputs are
# wrong by construction -- probes, never parity).  One pass per counter set.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/stpmc
for c in ${CFGS:-2 5}; do
  for v in ${VARIANTS:-base noacl nonat noipf2}; do
    lib=dataplane_amd/lib/libdpgpu.so
    [ "$v" != base ] && lib=dataplane_amd/lib/libdpgpu_$v.so
    d=gpurun_out/stpmc/c${c}_$v
    mkdir -p $d
    i=0
    for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      DP_BENCH_NOCHECK=1 DPGPU_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $d/p$i -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-host --no-flows --no-nat > $d/p$i.json 2> $d/p$i.err || { echo "PMC_FAIL C$c $v pass $i"; tail -5 $d/p$i.err; exit 1; }
    done
    echo "C$c $v $(python3 scripts/pmc_kernel.py $d/p1 $d/p2 | tr -s ' ' | tr '\n' ';')"
  done
done
echo STAGE_PMC_OK
