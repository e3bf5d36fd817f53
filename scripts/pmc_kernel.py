# Summarise rocprofv3 --pmc CSVs: per-dispatch mean of each counter for one
# kernel (default dp_pipeline_kernel<false, false, false, *>, the non-flow variant the metric times), over every pass directory given.
import csv
import glob
import sys
from collections import defaultdict


def summarise(dirs, kernel="dp_pipeline_kernel<false, false, false"):
    vals = defaultdict(lambda: defaultdict(float))
    for d in dirs:
        files = glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True)
        for row in (r for f in files for r in csv.DictReader(open(f))):
            if kernel not in row["Kernel_Name"]:
                continue
            vals[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    for k, v in sorted(summarise(sys.argv[1:]).items()):
        print(f"{k:40s} {v:18.1f}")
