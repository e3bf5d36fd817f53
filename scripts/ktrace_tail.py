"""Print the last N dispatches of a rocprofv3 kernel trace (kernel_trace.csv):
name, duration and the gap since the previous dispatch ended."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r['Start_Timestamp']))
tail = rows[-n:]
prev = None
for r in tail:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{r['Kernel_Name'][:60]:60s} dur_us={(e - s) / 1e3:9.1f} gap_us={gap:8.1f}")
    prev = e
