#!/bin/bash
# run-to-run spread of the config-2/3 bench lines on one box
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bv3_$r.log 2>&1 || { tail -20 gpurun_out/bv3_$r.log; exit 1; }
  echo "cfg3 run $r $(tail -1 gpurun_out/bv3_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bv2.log 2>&1 || { tail -20 gpurun_out/bv2.log; exit 1; }
echo "cfg2 $(tail -1 gpurun_out/bv2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["phases_ms_per_step"])')"
rocm-smi --showclocks 2>/dev/null | grep -i "sclk\|mclk" | head -4 || true
