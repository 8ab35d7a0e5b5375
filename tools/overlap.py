"""Occupancy of the config-5 split-LSQR iteration loop from a rocprofv3 kernel
trace: over the span of the fused split kernels, the
fraction of time in which both batch slices run a pass, a pass runs beside a
Dπ launch, only Dπ launches run, only one pass runs, or nothing runs (the
host's convergence read-backs).

  python tools/overlap.py DIR
"""
import csv
import glob
import os
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
ev = []
for r in csv.DictReader(open(path)):
    kn = r["Kernel_Name"]
    if "conic_fsplit_pass_kernel" in kn:
        kind = "pass"
    elif "conic_fsplit_dpi" in kn:
        kind = "dpi"
    else:
        continue
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
if not ev:
    sys.exit("no fused split kernels in the trace")
pts = sorted({t for s, e, _ in ev for t in (s, e)})
acc = {"both slices in a pass": 0, "pass beside Dπ": 0, "one pass alone": 0, "Dπ only": 0, "idle": 0}
ev.sort()
for a, b in zip(pts, pts[1:]):
    mid = (a + b) / 2
    act = [k for s, e, k in ev if s <= mid < e]
    npass, ndpi = act.count("pass"), act.count("dpi")
    key = ("both slices in a pass" if npass >= 2 else "pass beside Dπ" if npass and ndpi else
           "one pass alone" if npass else "Dπ only" if ndpi else "idle")
    acc[key] += b - a
tot = pts[-1] - pts[0]
print(f"{path}: fused split LSQR span {tot / 1e6:.2f} ms, {len(ev)} launches")
for k, v in acc.items():
    print(f"  {k:24s} {100.0 * v / tot:5.1f} %")
