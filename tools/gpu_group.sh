#!/bin/bash
# panel-group sweep (DOPT_LU_GROUP) on configs 2 and 3, after the GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_grp.log 2>&1 || { tail -30 gpurun_out/t_grp.log; exit 1; }
tail -1 gpurun_out/t_grp.log
for g in 0 2 3 4; do
  DOPT_LU_GROUP=$g timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bg2_$g.log 2>&1 || { tail -20 gpurun_out/bg2_$g.log; exit 1; }
  echo "cfg2 group=$g $(tail -1 gpurun_out/bg2_$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
for g in 0 4 3; do
  DOPT_LU_GROUP=$g timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bg3_$g.log 2>&1 || { tail -20 gpurun_out/bg3_$g.log; exit 1; }
  echo "cfg3 group=$g $(tail -1 gpurun_out/bg3_$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
