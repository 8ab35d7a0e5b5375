#!/bin/bash
# conic GPU parity tests, then a conic bench line: tools/gpu_conic_test.sh TAG [bench args...]
set -o pipefail
tag=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_conic_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tc_$tag.log 2>&1 || { tail -30 gpurun_out/tc_$tag.log; exit 1; }
tail -2 gpurun_out/tc_$tag.log
timeout -k 10 400 python bench.py "$@" > gpurun_out/bc_$tag.log 2>&1 || { tail -20 gpurun_out/bc_$tag.log; exit 1; }
tail -1 gpurun_out/bc_$tag.log
