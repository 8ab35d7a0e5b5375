# Sweep row groups of 16 vs 8 (DOPT_SYM_RH) on configs 2 and 6, with the NLP tests under RH=16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
DOPT_SYM_RH=16 TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_rh16.log && \
bash $J bench cfg2rh8 --steps 20 --warmup 3 --no-cpu-baseline && \
DOPT_SYM_RH=16 bash $J bench cfg2rh16 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg6rh8 --config 6 --steps 20 --warmup 3 --no-cpu-baseline && \
DOPT_SYM_RH=16 bash $J bench cfg6rh16 --config 6 --steps 20 --warmup 3 --no-cpu-baseline
