#!/bin/bash
# blocked-LU stream-chunk sweep: config 2 and 3 at DOPT_LU_STREAMS = 1..4, then GPU suite
set -o pipefail
mkdir -p gpurun_out
for s in 1 2 3 4; do
  DOPT_LU_STREAMS=$s timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bs2_$s.log 2>&1 || { tail -20 gpurun_out/bs2_$s.log; exit 1; }
  echo "cfg2 streams=$s $(tail -1 gpurun_out/bs2_$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
for s in 1 2; do
  DOPT_LU_STREAMS=$s timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bs3_$s.log 2>&1 || { tail -20 gpurun_out/bs3_$s.log; exit 1; }
  echo "cfg3 streams=$s $(tail -1 gpurun_out/bs3_$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_streams.log 2>&1 || { tail -30 gpurun_out/t_streams.log; exit 1; }
tail -2 gpurun_out/t_streams.log
