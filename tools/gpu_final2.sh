#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_final2.log 2>&1 || { tail -30 gpurun_out/t_final2.log; exit 1; }
tail -1 gpurun_out/t_final2.log
timeout -k 10 120 python tools/nccl_pipe_check.py > gpurun_out/nccl.log 2>&1 || { tail -20 gpurun_out/nccl.log; exit 1; }
tail -1 gpurun_out/nccl.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
