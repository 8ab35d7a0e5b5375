#!/bin/bash
# strip trailing-update sweep (DOPT_UPD_CT) on configs 2 and 3, parity first
set -o pipefail
mkdir -p gpurun_out
DOPT_UPD_CT=2 timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ct2.log 2>&1 || { tail -30 gpurun_out/t_ct2.log; exit 1; }
tail -1 gpurun_out/t_ct2.log
DOPT_UPD_CT=4 timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "blocked or cfg2 or ragged" > gpurun_out/t_ct4.log 2>&1 || { tail -30 gpurun_out/t_ct4.log; exit 1; }
tail -1 gpurun_out/t_ct4.log
for c in 1 2 4; do
  DOPT_UPD_CT=$c timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bc2_$c.log 2>&1 || { tail -20 gpurun_out/bc2_$c.log; exit 1; }
  echo "cfg2 ct=$c $(tail -1 gpurun_out/bc2_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
for c in 1 2 4; do
  DOPT_UPD_CT=$c timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bc3_$c.log 2>&1 || { tail -20 gpurun_out/bc3_$c.log; exit 1; }
  echo "cfg3 ct=$c $(tail -1 gpurun_out/bc3_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
