# Probe: the Q symmetry check overlapping the LU instead of the prepare kernel (DOPT_QSYM_LATE=1, no verdict), config 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
bash $J bench cfg2base --steps 20 --warmup 3 --no-cpu-baseline && \
DOPT_QSYM_LATE=1 bash $J bench cfg2late --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg2base2 --steps 20 --warmup 3 --no-cpu-baseline && \
DOPT_QSYM_LATE=1 bash $J bench cfg2late2 --steps 20 --warmup 3 --no-cpu-baseline
