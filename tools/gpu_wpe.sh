#!/bin/bash
# assembly kernel occupancy: waves-per-EU 5 (82 VGPRs) / 6 / 8, prebuilt variants in gpurun_var/
set -o pipefail
mkdir -p gpurun_out
L=diffopt.jl_amd/diffopt_amd/libdiffopt_mi355x.so
for w in 5 6 8 5 6 8; do
cp gpurun_var/lib_wpe$w.so $L
for cfg in 2 3; do
timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_wpe.log 2>&1 || { tail -20 gpurun_out/b_wpe.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/b_wpe.log').read().strip().splitlines()[-1]);print('cfg $cfg wpe $w', d['value'], d['roofline']['phases_ms_per_step'].get('qp_assemble'))"
done; done
for w in 6 8; do cp gpurun_var/lib_wpe$w.so $L
timeout -k 10 300 python -u -m pytest tests/test_qp_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_wpe.log 2>&1 || { tail -30 gpurun_out/t_wpe.log; exit 1; }
echo "wpe $w: $(tail -1 gpurun_out/t_wpe.log)"; done
