#!/bin/bash
# GPU suite, then config-2 bench for the product library and tuning variants ($VARIANTS)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_var.log 2>&1 || { tail -30 gpurun_out/t_var.log; exit 1; }
tail -1 gpurun_out/t_var.log
for v in "" ${VARIANTS}; do
  DOPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bv_$v.log 2>&1 || { tail -20 gpurun_out/bv_$v.log; exit 1; }
  echo "variant=[$v] $(tail -1 gpurun_out/bv_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
