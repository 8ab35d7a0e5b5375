"""Compact view of a rocprofv3 kernel_stats.csv (a file, or the directory
rocprofv3 -d wrote): short name, calls, total ms over the whole profiled run
(`total_ms`; with `per` = the number of bench steps incl. warmup given, the
total divided by it, `ms_per_step`), avg µs per launch, share."""
import csv
import glob
import os
import re
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = sorted(glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True))[0]
per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
print(path)
for r in rows[:20]:
    name = r["Name"]
    m = re.search(r"(\w+(?:<[^>]*>)?)\(", name)
    short = m.group(1) if m else name[:60]
    col = "ms_per_step" if len(sys.argv) > 2 else "total_ms"
    print(f"{short[:48]:48s} calls={int(r['Calls']):5d} {col}={float(r['TotalDurationNs'])/1e6/per:8.4f} "
          f"avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
