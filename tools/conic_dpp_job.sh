set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
TEST_PATHS=tests/test_conic_gpu.py bash $J test && cp gpurun_out/test.log gpurun_out/test_conic.log && \
bash $J bench cfg5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J bench cfg4 --config 4 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J prof cfg5 --config 5 --steps 2 --warmup 1 && \
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" && \
timeout -s KILL 300 rocprofv3 --pmc $SQ -d gpurun_out/sq_cfg5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 5 --steps 1 --warmup 1 > gpurun_out/sq_cfg5.log 2>&1
