# Small path with one copy each way: its GPU tests, then the drop-in latency
# of this build and of the HEAD build (variants/libdiffopt_prev.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_qp_small_gpu.py tests/test_qp_gpu.py tests/test_lhs_solve_gpu.py > gpurun_out/small_io_tests.log 2>&1 || { tail -30 gpurun_out/small_io_tests.log; exit 1; }
tail -2 gpurun_out/small_io_tests.log
for r in 1; do
  DOPT_LIB=diffopt.jl_amd/diffopt_amd/variants/libdiffopt_prev.so timeout -k 10 300 python3 -u tools/bench_dropin.py > gpurun_out/dropin_prev_$r.jsonl 2>/dev/null || exit 1
  timeout -k 10 300 python3 -u tools/bench_dropin.py > gpurun_out/dropin_base_$r.jsonl 2>/dev/null || exit 1
done
