# Round 5: full GPU suite, then the config-2 bench line and its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_${TAG:-r05}.log && \
bash $J prof ${TAG:-r05}cfg2 --steps 20 --warmup 3
