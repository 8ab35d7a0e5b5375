#!/bin/bash
# solve2 workgroup order: parity with DOPT_SOLVE_ILV=1, then config 2/3 benches both ways
set -o pipefail
mkdir -p gpurun_out
DOPT_SOLVE_ILV=1 timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_ilv.log 2>&1 || { tail -30 gpurun_out/t_ilv.log; exit 1; }
tail -1 gpurun_out/t_ilv.log
for cfg in 2 3; do for ilv in 0 1 0 1; do
DOPT_SOLVE_ILV=$ilv timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_ilv.log 2>&1 || { tail -20 gpurun_out/b_ilv.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/b_ilv.log').read().strip().splitlines()[-1]);print('cfg $cfg ilv $ilv', d['value'], d['roofline']['phases_ms_per_step'].get('qp_solve'))"
done; done
