#!/usr/bin/env python3
"""Per-kernel totals of rocprofv3 --pmc counters: sum of each counter over a
kernel's dispatches, divided by its dispatch count (per-launch average).

  python tools/pmc_kernels.py <pmc_dir> [name_fragment ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    frags = sys.argv[2:]
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row.get("Kernel_Name", "")
                short = kn.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:48]
                if frags and not any(x in kn for x in frags):
                    continue
                tot[short][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[short].add(row.get("Dispatch_Id"))
    counters = sorted({c for v in tot.values() for c in v})
    print(f"{'kernel':48s} {'launches':>8s} " + " ".join(f"{c:>24s}" for c in counters))
    for k in sorted(tot, key=lambda k: -sum(tot[k].values())):
        n = len(disp[k])
        print(f"{k:48s} {n:8d} " + " ".join(f"{tot[k].get(c, 0.0) / n:24.0f}" for c in counters))


if __name__ == "__main__":
    main()
