#!/bin/bash
# panel change check: QP GPU tests, config 2/3 bench, panel stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_pan.log 2>&1 || { tail -30 gpurun_out/t_pan.log; exit 1; }
tail -1 gpurun_out/t_pan.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bp2.log 2>&1 || { tail -20 gpurun_out/bp2.log; exit 1; }
echo "cfg2 $(tail -1 gpurun_out/bp2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bp3.log 2>&1 || { tail -20 gpurun_out/bp3.log; exit 1; }
echo "cfg3 $(tail -1 gpurun_out/bp3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
timeout -k 10 100 python tools/stamps_blocked.py 2 1024 2>&1 | grep -v amdgpu.ids
