"""Print the top kernels of a rocprofv3 --stats CSV (run_kernel_stats.csv)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for r in rows[:n]:
    print(f"{r['Name'][:62]:62s} calls={r['Calls']:>5} total_ms={float(r['TotalDurationNs'])/1e6:9.2f} "
          f"avg_us={float(r['AverageNs'])/1e3:9.1f} max_us={float(r['MaxNs'])/1e3:9.1f}")
