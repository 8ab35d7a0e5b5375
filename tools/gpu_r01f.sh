#!/bin/bash
# r01f: GPU suite + config-2 bench (fused vs blocked route) + rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 3 > gpurun_out/b2.log 2>&1 || { tail -20 gpurun_out/b2.log; exit 1; }
tail -1 gpurun_out/b2.log
DOPT_FAST_MAX=0 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b2_blocked.log 2>&1 || { tail -20 gpurun_out/b2_blocked.log; exit 1; }
tail -1 gpurun_out/b2_blocked.log
export TMPDIR=/tmp
DOPT_FAST_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b2blk -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_b2blk.log 2>&1 || { tail -20 gpurun_out/prof_b2blk.log; exit 1; }
find gpurun_out/prof_b2blk -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
