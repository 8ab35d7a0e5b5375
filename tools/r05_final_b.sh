# Round-5 closing refresh, part B: config 2 interior-point, config 3 (+ trace,
# PMC), config 3 interior-point
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J bench cfg2lam --lam-eps 1e-9 --no-cpu-baseline \
 && PMC_SUFFIX=@lam bash $J pmc cfg2lam --lam-eps 1e-9 --steps 3 --warmup 1 \
 && bash $J bench cfg3 --config 3 --steps 5 --warmup 2 \
 && bash $J prof cfg3 --config 3 --steps 3 --warmup 1 \
 && PMC_SUFFIX=@cfg3 bash $J pmc cfg3 --config 3 --steps 2 --warmup 1 \
 && bash $J bench cfg3lam --config 3 --lam-eps 1e-9 --steps 2 --warmup 1 --no-cpu-baseline
