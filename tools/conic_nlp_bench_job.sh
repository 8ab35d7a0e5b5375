set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J bench cfg4 --config 4 --steps 2 --warmup 1 --no-cpu-baseline && bash $J bench cfg4w --config 4 --conic-variant wellcond --steps 3 --warmup 1 --no-cpu-baseline && bash $J bench cfg5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && bash $J prof cfg5 --config 5 --steps 2 --warmup 1 && bash $J bench cfg6 --config 6 --steps 10 --warmup 2 --no-cpu-baseline
