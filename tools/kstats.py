"""Compact view of a rocprofv3 kernel_stats.csv: short name, calls, total ms,
avg µs, share; `per` = number of bench steps (incl. warmup) to divide by."""
import csv, re, sys
path = sys.argv[1]
per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
for r in rows[:14]:
    name = r["Name"]
    m = re.search(r"(\w+(?:<[^>]*>)?)\(", name)
    short = m.group(1) if m else name[:60]
    print(f"{short[:48]:48s} calls={int(r['Calls']):5d} ms/step={float(r['TotalDurationNs'])/1e6/per:8.4f} "
          f"avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
