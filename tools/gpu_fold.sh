#!/bin/bash
# narrow-update fold: QP parity, config 2/3 with and without (DOPT_NARROW_FOLD)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_fold.log 2>&1 || { tail -30 gpurun_out/t_fold.log; exit 1; }
tail -1 gpurun_out/t_fold.log
for f in 1 0; do
  DOPT_NARROW_FOLD=$f timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bf2_$f.log 2>&1 || { tail -20 gpurun_out/bf2_$f.log; exit 1; }
  echo "cfg2 fold=$f $(tail -1 gpurun_out/bf2_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
  DOPT_NARROW_FOLD=$f timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bf3_$f.log 2>&1 || { tail -20 gpurun_out/bf3_$f.log; exit 1; }
  echo "cfg3 fold=$f $(tail -1 gpurun_out/bf3_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
