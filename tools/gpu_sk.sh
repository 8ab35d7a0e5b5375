#!/bin/bash
# conic config-5 split LSQR: SPLIT_K tuning variants (DOPT_LIB_VARIANT)
set -o pipefail
mkdir -p gpurun_out
for v in "" sk4 sk6 sk12 sk16; do
  DOPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bsk_$v.log 2>&1 || { tail -20 gpurun_out/bsk_$v.log; exit 1; }
  echo "variant=[$v] $(tail -1 gpurun_out/bsk_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
done
