# LU-mode A/B on config 2 / 3 (bench lines) + the QP parity subset
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J bench cfg2 --no-cpu-baseline || exit 1
DOPT_LCOL_PF=0 bash $J bench cfg2nopf --no-cpu-baseline || exit 1
bash $J bench cfg3 --config 3 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
DOPT_LCOL_PF=0 bash $J bench cfg3nopf --config 3 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py" bash $J test
