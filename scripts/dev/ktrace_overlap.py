"""Per flow-burst launch of a rocprofv3 kernel trace: each NAT-pass kernel's
[start, end) in us from the first pass's start -- to see what the side
stream's replay overlaps."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
SHORT = [("dp_pipeline_kernel<true, false, true", "replay"), ("dp_pipeline_kernel<true, true, true", "replay"),
         ("dp_pipeline_kernel<true", "first"), ("dp_nat_resolve<true>", "resolve1"), ("dp_nat_resolve<false>", "resolve"),
         ("dp_nat_lane_plan", "plan"), ("dp_nat_lane_end", "lane_end"), ("dp_nat_lane(", "lane"), ("dp_nat_pairs", "pairs"),
         ("dp_flow_fixup", "fixup"), ("dp_flow_apply", "apply"), ("dp_bits_", "bits"), ("dp_nat_mark", "mark"),
         ("dp_nat_prep", "prep"), ("dp_nat_cross", "cross"), ("dp_nat_admit", "admit"), ("dp_stats_reduce", "stats")]
t0 = None
out = []
for r in rows:
    n = r['Kernel_Name']
    a, b = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = next((s for p, s in SHORT if p in n), None)
    if name is None:
        continue
    if name == "first":
        t0 = a
        out = []
    if t0 is None:
        continue
    out.append(f"{name}[{(a - t0) / 1e3:.0f},{(b - t0) / 1e3:.0f}]")
    if name == "apply":
        print(" ".join(out))
        t0 = None
