#!/bin/bash
# conic tuning pass (GPU box helper): parity tests, config 4/5 lines, variant
# libraries (DOPT_LIB_VARIANT), rocprofv3 kernel stats of config 5
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conic_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1 || { tail -30 gpurun_out/tc.log; exit 1; }
tail -1 gpurun_out/tc.log
for v in "" ${VARIANTS}; do
  DOPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --config 5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bc_c5_$v.log 2>&1 || { tail -20 gpurun_out/bc_c5_$v.log; exit 1; }
  echo "c5 $v"; tail -1 gpurun_out/bc_c5_$v.log | cut -c1-900
done
timeout -k 10 200 python bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bc_c4.log 2>&1 || { tail -20 gpurun_out/bc_c4.log; exit 1; }
echo c4; tail -1 gpurun_out/bc_c4.log | cut -c1-900
bash tools/prof_kernels.sh c5 --config 5 --steps 1 --warmup 1
