#!/bin/bash
# rocprofv3 kernel-trace summary of one bench configuration (GPU box helper).
#   tools/prof_kernels.sh TAG [bench.py args...]
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- \
  python bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
tail -1 gpurun_out/prof_$tag.log
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-60:]
    print(f'{name:60s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:10.1f} tot_ms={float(r["TotalDurationNs"])/1e6:9.2f} {float(r["Percentage"]):5.1f}%')
PY
