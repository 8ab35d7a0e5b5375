#!/bin/bash
# round-1 closing check: gpu parity suite, default bench line, rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r01j.log 2>&1 || { tail -30 gpurun_out/t_r01j.log; exit 1; }
tail -1 gpurun_out/t_r01j.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r01j.log 2>&1 || { tail -20 gpurun_out/smoke_r01j.log; exit 1; }
tail -1 gpurun_out/smoke_r01j.log
bash tools/run_bench_prof.sh r01j 10
