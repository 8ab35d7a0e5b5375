# small-path kernel variants: its GPU tests (this build), then the drop-in
# latency of the HEAD build, this build and the rcp variant, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_qp_small_gpu.py \
  > gpurun_out/small_ab_tests.log 2>&1 || { tail -30 gpurun_out/small_ab_tests.log; exit 1; }
tail -1 gpurun_out/small_ab_tests.log
DOPT_LIB=diffopt.jl_amd/diffopt_amd/variants/libdiffopt_rcp.so timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_qp_small_gpu.py \
  > gpurun_out/small_ab_tests_rcp.log 2>&1 || { tail -30 gpurun_out/small_ab_tests_rcp.log; exit 1; }
tail -1 gpurun_out/small_ab_tests_rcp.log
VARIANT=rcp bash tools/r05_dropin_ab.sh
