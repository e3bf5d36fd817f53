"""One flow-burst launch of a rocprofv3 kernel trace: the dispatches from the
k-th last dp_flow_apply back to the previous one (per kernel: duration and the
gap before it), and the launch's span."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows.sort(key=lambda r: int(r['Start_Timestamp']))
ends = [i for i, r in enumerate(rows) if 'dp_flow_apply' in r['Kernel_Name']]
e = ends[-k]
s = ends[-k - 1] + 1
while 'rocclr' in rows[s]['Kernel_Name']:
    s += 1
prev = None
tot = 0
for r in rows[s:e + 1]:
    a, b = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (a - prev) / 1e3 if prev is not None else 0.0
    tot += b - a
    print(f"{r['Kernel_Name'][:64]:64s} dur_us={(b - a) / 1e3:8.1f} gap_us={gap:7.1f}")
    prev = b
span = int(rows[e]['End_Timestamp']) - int(rows[s]['Start_Timestamp'])
print(f"span_us={span / 1e3:.1f} busy_us={tot / 1e3:.1f} dispatches={e + 1 - s}")
