set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS=tests/test_conic_gpu.py bash $J test && cp gpurun_out/test.log gpurun_out/test_conic.log && \
bash $J bench cfg4 --config 4 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J bench cfg4w --config 4 --conic-variant wellcond --steps 3 --warmup 1 --no-cpu-baseline && \
bash $J bench cfg5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline
