#!/bin/bash
# GPU suite + config-2 bench + rocprof kernel stats (tag = $1)
set -o pipefail
tag=${1:-q}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { tail -30 gpurun_out/t_$tag.log; exit 1; }
tail -2 gpurun_out/t_$tag.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_$tag.log 2>&1 || { tail -20 gpurun_out/b_$tag.log; exit 1; }
tail -1 gpurun_out/b_$tag.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
python tools/kstats.py gpurun_out/prof_$tag/run_kernel_stats.csv 6
