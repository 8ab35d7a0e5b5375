#!/bin/bash
# swizzled-LDS trailing-update variant: parity, then config 2/3 against the product build
set -o pipefail
mkdir -p gpurun_out
DOPT_LIB_VARIANT=swz timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_swz.log 2>&1 || { tail -30 gpurun_out/t_swz.log; exit 1; }
tail -1 gpurun_out/t_swz.log
for v in "" swz; do
  DOPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bw2_$v.log 2>&1 || { tail -20 gpurun_out/bw2_$v.log; exit 1; }
  echo "cfg2 [$v] $(tail -1 gpurun_out/bw2_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
  DOPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bw3_$v.log 2>&1 || { tail -20 gpurun_out/bw3_$v.log; exit 1; }
  echo "cfg3 [$v] $(tail -1 gpurun_out/bw3_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
