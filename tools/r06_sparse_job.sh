# Round 6: the sparse route (QP + conic) and the conic suite (the persistent
# LSQR kernel is now templated on its A products), then the sparse bench lines
# (configs 7 / 8) and the config-2 line with the step-level roofline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS="tests/test_sparse_gpu.py tests/test_conic_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_sparse_conic.log && \
bash $J bench cfg7 --config 7 --steps 5 --warmup 1 && \
bash $J bench cfg8 --config 8 --steps 5 --warmup 1 && \
bash $J bench cfg2 --no-cpu-baseline
