# NLP reverse outputs by 8-lane column groups, vectorised J scan: NLP tests, config-6 bench and kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS="tests/test_nlp_gpu.py tests/test_model_api_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_nlpout.log && \
bash $J bench cfg6 --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J prof cfg6 --config 6 --steps 10 --warmup 2
