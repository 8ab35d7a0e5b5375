#!/bin/bash
# conic parity + config 4/5 bench lines (tag $1) + config-4 rocprof kernel stats
set -o pipefail
tag=${1:-r01f}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conic_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/tc_$tag.log 2>&1 || { tail -30 gpurun_out/tc_$tag.log; exit 1; }
tail -1 gpurun_out/tc_$tag.log
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_${tag}_c4.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c4.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c4.log
timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${tag}_c5.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c5.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c5.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c4 -o run --output-format csv -- python bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${tag}_c4.log 2>&1 || { tail -20 gpurun_out/prof_${tag}_c4.log; exit 1; }
python tools/kstats.py gpurun_out/prof_${tag}_c4/run_kernel_stats.csv 2
