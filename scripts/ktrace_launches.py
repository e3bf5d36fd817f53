"""Every flow-burst launch of a rocprofv3 kernel trace (dispatches from a
first-pass dp_pipeline_kernel to the next dp_flow_apply): span and the
durations of its main kernels, one line per launch in order."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
KEYS = [("first", "dp_pipeline_kernel<true, false, false"), ("first", "dp_pipeline_kernel<true, true, false"),
        ("mark", "dp_nat_mark"), ("prep", "dp_nat_prep"), ("cross", "dp_nat_cross"), ("resolve1", "dp_nat_resolve<true>"),
        ("resolve", "dp_nat_resolve<false>"), ("plan", "dp_nat_lane_plan"), ("lane", "dp_nat_lane("),
        ("pairs", "dp_nat_pairs"), ("replay", "dp_pipeline_kernel<true, false, true"),
        ("replay", "dp_pipeline_kernel<true, true, true")]
cur = None
k = 0
for r in rows:
    n = r['Kernel_Name']
    a, b = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if n.startswith('void (anonymous namespace)::dp_pipeline_kernel<true') and ', false,' in n.split('<')[1][:20] and cur is None:
        cur = {"t0": a}
    if cur is None:
        continue
    for key, pat in KEYS:
        if pat in n:
            cur[key] = cur.get(key, 0) + (b - a) / 1e3
    if 'dp_flow_apply' in n:
        k += 1
        span = (b - cur.pop("t0")) / 1e3
        print(f"{k:3d} span {span:8.1f} us  " + "  ".join(f"{x} {cur[x]:.1f}" for x in
              ["first", "mark", "prep", "cross", "resolve1", "resolve", "plan", "lane", "pairs", "replay"] if x in cur))
        cur = None
