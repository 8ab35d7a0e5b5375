# LU-mode A/B on config 2 / 3 (bench lines) + the QP parity subset under the persistent mode
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_job.sh bench cfg2 --no-cpu-baseline || exit 1
DOPT_LPERSIST=1 bash tools/gpu_job.sh bench cfg2persist --no-cpu-baseline || exit 1
DOPT_LSLICE=2 bash tools/gpu_job.sh bench cfg2slice --no-cpu-baseline || exit 1
DOPT_LPERSIST=1 TEST_PATHS="tests/test_qp_gpu.py" bash tools/gpu_job.sh test -k "config or fixture or left" || exit 1
bash tools/gpu_job.sh bench cfg3 --config 3 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
DOPT_LPERSIST=1 bash tools/gpu_job.sh bench cfg3persist --config 3 --steps 5 --warmup 2 --no-cpu-baseline
