"""Per-kernel SQ counter ratios from a rocprofv3 --pmc run.

    python tools/sq_summary.py gpurun_out/sq_cfg5 [name-fragment ...]

Sums every counter over the dispatches of each kernel (by name, template
arguments dropped) and prints each counter as a fraction of SQ_WAVE_CYCLES
(the wave-cycles the kernel's waves were resident), plus the dispatch count.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main(d, frags):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = re.sub(r"<.*", "", row.get("Kernel_Name", "")).split("(")[0]
                if frags and not any(fr in kn for fr in frags):
                    continue
                acc[kn][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[kn].add(row.get("Dispatch_Id"))
    names = sorted({c for v in acc.values() for c in v})
    other = [c for c in names if c != "SQ_WAVE_CYCLES"]
    print(f"{'kernel':34s} {'disp':>6s} " + " ".join(f"{c.replace('SQ_', '').lower()[:14]:>14s}" for c in other))
    for kn, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1.0
        print(f"{kn[-34:]:34s} {len(disp[kn]):6d} " + " ".join(f"{v.get(c, 0) / wc:14.3f}" for c in other))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
