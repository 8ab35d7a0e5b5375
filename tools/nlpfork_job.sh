# NLP: H symmetry check beside the reduction prep (second stream) — NLP / model tests, config-6 bench twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS="tests/test_nlp_gpu.py tests/test_model_api_gpu.py tests/test_lhs_solve_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_nlpfork.log && \
bash $J bench cfg6f --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg6f2 --config 6 --steps 20 --warmup 3 --no-cpu-baseline
