#!/usr/bin/env python3
"""Counter calibration per access width: reads the two rocprofv3 passes of
tools/probe/pmc_cal (every kernel streams exactly 1 GiB with one access width)
and writes counter-bytes ÷ streamed-bytes per kernel and counter.

  python tools/pmc_calibrate.py <fetch_dir> <write_dir> profiles/pmc_calibration.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

STREAMED = 1 << 30
KERNELS = {"rd<float>": "load 4 B/lane", "rd<double>": "load 8 B/lane", "rd16": "load 16 B/lane",
           "rd8_rows": "load 8 B/lane, 4 rows x 128 B (LU tile pattern)", "wr<double>": "store 8 B/lane",
           "wr16": "store 16 B/lane", "wr<float>": "store 4 B/lane"}


def counter(d, name):
    out = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != name:
                    continue
                for frag, label in KERNELS.items():
                    if row["Kernel_Name"].startswith(("void " + frag, frag)):
                        out[label] += float(row["Counter_Value"]) * 1024   # KB → B
    return out


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch, write = counter(fdir, "FETCH_SIZE"), counter(wdir, "WRITE_SIZE")
    res = {"streamed_bytes_per_kernel": STREAMED,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE on tools/probe/pmc_cal, separate passes",
           "ratio_counter_to_streamed": {k: {"FETCH_SIZE": fetch.get(k, 0.0) / STREAMED,
                                             "WRITE_SIZE": write.get(k, 0.0) / STREAMED}
                                         for k in KERNELS.values()}}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
