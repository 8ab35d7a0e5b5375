#!/bin/bash
# bench + rocprofv3 kernel-trace summary (GPU box helper)
set -o pipefail
tag=${1:-r01}
steps=${2:-10}
timeout -k 10 400 python bench.py --steps $steps --warmup 2 --cpu-seconds ${CPU_SECONDS:-5} > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-250
