# NLP reduction pairs with 512-thread workgroups (DOPT_RED_TPB=512) vs 256: NLP tests under 512, config-6 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
DOPT_RED_TPB=512 TEST_PATHS="tests/test_nlp_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_red512.log && \
bash $J bench cfg6t256 --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
DOPT_RED_TPB=512 bash $J bench cfg6t512 --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg6t256b --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
DOPT_RED_TPB=512 bash $J bench cfg6t512b --config 6 --steps 20 --warmup 3 --no-cpu-baseline
