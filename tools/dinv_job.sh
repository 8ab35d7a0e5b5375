# P-symmetric sweeps with the diagonal inverses staged in LDS (one block ahead): QP / NLP tests, configs 2, 3, 6, config-2 trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py tests/test_multi_rhs_gpu.py tests/test_lhs_solve_gpu.py tests/test_model_api_gpu.py tests/test_params_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_dinv.log && \
bash $J bench cfg2 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg6 --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg3 --config 3 --steps 3 --warmup 1 --no-cpu-baseline && \
bash $J prof cfg2 --steps 20 --warmup 3
