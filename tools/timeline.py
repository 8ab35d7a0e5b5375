"""Per-dispatch timeline of one bench step from a rocprofv3 kernel trace (the
directory `rocprofv3 --kernel-trace -d DIR` wrote): every kernel of the window
that starts at the K-th-from-last dispatch of `first` (default: the prepare
kernel, the first launch of a QP step), with its start offset, duration and
queue, so the critical chain across the engine's two streams can be read off.

  python tools/timeline.py DIR [first_kernel_substring] [steps_from_end]
"""
import csv
import glob
import os
import re
import sys

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "qp_prep_kernel"
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
if os.path.isdir(path):
    path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(name):
    m = re.search(r"(\w+(?:<[^>]*>)?)\(", name)
    return (m.group(1) if m else name)[:40]


starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
if len(starts) < back + 1:
    sys.exit(f"fewer than {back + 1} dispatches of {first}")
i0, i1 = starts[-back - 1], starts[-back]
t0 = int(rows[i0]["Start_Timestamp"])
end = t0
print(f"{path}: step window of {i1 - i0} dispatches")
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    end = max(end, e)
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    print(f"{(s - t0) / 1e3:9.1f} us  +{(e - s) / 1e3:8.1f} us  q{q:>3s}  {short(r['Kernel_Name'])}")
nxt = int(rows[i1]["Start_Timestamp"])
print(f"step: last kernel ends at {(end - t0) / 1e3:.1f} us, next step starts at {(nxt - t0) / 1e3:.1f} us")
