# Sensitivity of the C2 kernel time to table sizes (where the time goes):
# the default tables, then one table shrunk at a time.  Kernel time only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sens
run() {  # name, extra bench args
  timeout -k 10 240 python3 bench.py --config ${CFG:-2} --no-cpu --no-host --no-flows --steps 10 --warmup 3 $2 > gpurun_out/sens/$1.json 2> gpurun_out/sens/$1.err || { echo "FAIL $1"; tail -3 gpurun_out/sens/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sens/$1.json'));print('$1', d['value'], d['roofline']['kernel_ms'], d['roofline']['kernel_ms_median'])"
}
run base ""
run routes64k "--routes-v4 60000"
run routes200k "--routes-v4 200000"
run acl1k "--acl 1000"
run nat32 "--nat 32"
run base2 ""
