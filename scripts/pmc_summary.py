"""Summarise rocprofv3 --pmc CSVs of dp_pipeline_kernel<false, false, ...> (the non-flow, no-meta variant
the metric times; the bench flow-table leg launches the <true> variant): per-dispatch mean of
every counter (summed over dimensions), plus derived ratios.
    python scripts/pmc_summary.py gpurun_out/pmc [n_packets]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    npk = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "dp_pipeline_kernel<false, false" not in r.get("Kernel_Name", ""):
                continue
            per[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    tot, cnt = defaultdict(float), defaultdict(int)
    for d in per.values():
        for k, v in d.items():
            tot[k] += v
            cnt[k] += 1
    m = {k: tot[k] / cnt[k] for k in tot}
    out = {"per_dispatch": {k: round(v, 1) for k, v in sorted(m.items())}}
    dv = {}
    if "SQ_WAVES" in m:
        w = m["SQ_WAVES"]
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY",
                  "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY"):
            if k in m:
                dv[k + "_per_wave"] = round(m[k] / w, 1)
    if "FETCH_SIZE" in m:
        dv["fetch_bytes_per_pkt_x2"] = round(2 * m["FETCH_SIZE"] * 1024 / npk, 1)
    if "WRITE_SIZE" in m:
        dv["write_bytes_per_pkt"] = round(m["WRITE_SIZE"] * 1024 / npk, 1)
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        dv["l2_hit"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
    out["derived"] = dv
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
