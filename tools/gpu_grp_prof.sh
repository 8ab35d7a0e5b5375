#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for g in 0 4; do
DOPT_LU_GROUP=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g$g -o run --output-format csv -- python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_g$g.log 2>&1 || { tail -20 gpurun_out/prof_g$g.log; exit 1; }
echo "== group $g"; python tools/kstats.py gpurun_out/prof_g$g/run_kernel_stats.csv 3
done
