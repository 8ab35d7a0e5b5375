#!/bin/bash
# conic config-4 LSQR: PAIR_NC tuning variants (DOPT_LIB_VARIANT)
set -o pipefail
mkdir -p gpurun_out
for v in "" nc3 nc4 nc1; do
  DOPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bnc_$v.log 2>&1 || { tail -20 gpurun_out/bnc_$v.log; exit 1; }
  echo "variant=[$v] $(tail -1 gpurun_out/bnc_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
done
