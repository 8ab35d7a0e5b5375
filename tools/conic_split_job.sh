set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
TEST_PATHS=tests/test_conic_gpu.py bash $J test && cp gpurun_out/test.log gpurun_out/test_fused.log && \
DOPT_SPLIT_FUSE=0 TEST_PATHS=tests/test_conic_gpu.py bash $J test -k "split or config5 or large_psd" && \
bash $J bench cfg5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
DOPT_SPLIT_FUSE=0 bash $J bench cfg5nofuse --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
DOPT_SPLIT_NW=8 bash $J bench cfg5nw8 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J prof cfg5 --config 5 --steps 2 --warmup 1
