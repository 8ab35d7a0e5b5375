# NLP column tiles: no δ load / identity term for strictly-lower entries — NLP tests, config-6 bench twice, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS="tests/test_nlp_gpu.py tests/test_lhs_solve_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_nlplower.log && \
bash $J bench cfg6l --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg6l2 --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J prof cfg6l --config 6 --steps 10 --warmup 2
