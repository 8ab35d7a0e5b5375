set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
DOPT_PARITY_CALIBRATE=1 TEST_PATHS=tests/test_conic_gpu.py bash $J test && cp gpurun_out/test.log gpurun_out/test_conic.log && cp gpurun_out/parity.jsonl gpurun_out/parity_conic.jsonl && \
TEST_PATHS="tests/test_nlp_gpu.py tests/test_qp_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_nlp_qp.log && \
bash $J bench cfg4 --config 4 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J bench cfg4w --config 4 --conic-variant wellcond --steps 3 --warmup 1 --no-cpu-baseline && \
bash $J bench cfg5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J bench cfg6 --config 6 --steps 10 --warmup 2 --no-cpu-baseline && \
bash $J bench cfg2 --steps 20 --warmup 3 --no-cpu-baseline
