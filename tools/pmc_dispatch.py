"""Per-dispatch HBM traffic of the last bench step from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; gfx950: FETCH_SIZE ×2, tools/pmc_summary.py):
every kernel from the last dispatch of `first` on, in order.

  python tools/pmc_dispatch.py <fetch_dir> <write_dir> [first_kernel_substring]
"""
import csv
import glob
import os
import re
import sys


def load(d, counter):
    path = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
    rows = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        rows[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0)
    return rows


def short(name):
    m = re.search(r"(\w+(?:<[^>]*>)?)\(", name)
    return (m.group(1) if m else name)[:44]


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
first = sys.argv[3] if len(sys.argv) > 3 else "qp_prep_kernel"
fids = sorted(fetch)
wids = sorted(write)
fs = [i for i in fids if first in fetch[i][0]]
ws = [i for i in wids if first in write[i][0]]
fwin = [i for i in fids if i >= fs[-2]][: len([i for i in fids if fs[-2] <= i < fs[-1]])]
wwin = [i for i in wids if i >= ws[-2]][: len(fwin)]
tf = tw = 0.0
for a, b in zip(fwin, wwin):
    nf, vf = fetch[a]
    nw, vw = write[b]
    assert short(nf) == short(nw), (nf, nw)
    tf += 2 * vf
    tw += vw
    print(f"{short(nf):44s}  read {2 * vf / 1e6:9.1f} MB  write {vw / 1e6:9.1f} MB")
print(f"{'step total':44s}  read {tf / 1e6:9.1f} MB  write {tw / 1e6:9.1f} MB")
