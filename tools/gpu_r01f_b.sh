#!/bin/bash
# solve workgroup-size variant on config 2; conic bench lines (configs 4, 5) with CPU baselines
set -o pipefail
mkdir -p gpurun_out
for v in "" pt256; do
  DOPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bv_$v.log 2>&1 || { tail -20 gpurun_out/bv_$v.log; exit 1; }
  echo "variant=[$v] $(tail -1 gpurun_out/bv_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_r01f_c4.log 2>&1 || { tail -20 gpurun_out/bench_r01f_c4.log; exit 1; }
tail -1 gpurun_out/bench_r01f_c4.log
timeout -k 10 300 python bench.py --config 5 --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_r01f_c5.log 2>&1 || { tail -20 gpurun_out/bench_r01f_c5.log; exit 1; }
tail -1 gpurun_out/bench_r01f_c5.log
