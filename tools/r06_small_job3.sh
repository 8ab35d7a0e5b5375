#!/bin/bash
# small path A/B: the probe (TRSM columns contiguous per wave, panel v_rcp),
# the small-path GPU tests, then the drop-in latency of head / copy-in-copy-out
# I/O (variant copyio) / step-by-step forward sweeps (variant fwdsteps), two
# rounds, and one rocprofv3 kernel trace of head
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=diffopt.jl_amd/diffopt_amd/variants
rm -f gpurun_out/small_ab.txt
for v in blk blk_st; do
  echo "== $v" >> gpurun_out/small_ab.txt
  timeout -k 10 60 tools/probebin_blk/small_probe_$v >> gpurun_out/small_ab.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_qp_small_gpu.py tests/test_qp_gpu.py tests/test_model_api_gpu.py tests/test_lhs_solve_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/test_small.log 2>&1 || exit 1
for r in 1 2; do
  for v in head; do
    lib=""; [ $v != head ] && lib=$V/libdiffopt_$v.so
    echo "== $v round $r" >> gpurun_out/small_ab.txt
    DOPT_LIB=$lib timeout -k 10 300 python3 -u tools/bench_dropin.py --reps 30 2>/dev/null >> gpurun_out/small_ab.txt || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dropin3 -o run --output-format csv \
  -- python3 tools/bench_dropin.py --reps 30 > gpurun_out/prof_dropin3.log 2>&1 \
 && python3 tools/kstats.py gpurun_out/prof_dropin3 > gpurun_out/dropin3_kstats.txt
cat gpurun_out/small_ab.txt | cut -c1-420; grep qp_small gpurun_out/dropin3_kstats.txt; tail -2 gpurun_out/test_small.log
