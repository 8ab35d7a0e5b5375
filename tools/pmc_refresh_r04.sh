# Round-4 PMC refresh: HBM bytes per launch (FETCH_SIZE / WRITE_SIZE passes) of
# the QP headline workloads and the two workloads whose `traffic` was null in r03
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J pmc cfg2 --steps 3 --warmup 1 \
 && PMC_SUFFIX=@lam bash $J pmc cfg2lam --lam-eps 1e-9 --steps 3 --warmup 1 \
 && PMC_SUFFIX=@cfg3 bash $J pmc cfg3 --config 3 --steps 2 --warmup 1 \
 && PMC_SUFFIX=@cfg3@lam bash $J pmc cfg3lam --config 3 --lam-eps 1e-9 --steps 1 --warmup 1 \
 && PMC_SUFFIX=@wellcond bash $J pmc cfg4w --config 4 --conic-variant wellcond --steps 2 --warmup 1 \
 && bash $J prof cfg2 --steps 10 --warmup 2
