set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py tests/test_multi_rhs_gpu.py tests/test_lhs_solve_gpu.py tests/test_model_api_gpu.py tests/test_params_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_sym.log && \
bash $J bench cfg6 --config 6 --steps 10 --warmup 2 --no-cpu-baseline && \
bash $J bench cfg2 --steps 20 --warmup 3 --no-cpu-baseline
