# Round-end refresh: parity suite, smoke, every bench line (CPU baselines on
# the N=1 headline lines), kernel stats and PMC traffic of the QP headline
# configs (outputs under gpurun_out/)
set -o pipefail
J=tools/gpu_job.sh
bash $J test && bash $J smoke \
 && bash $J bench cfg2 && bash $J prof cfg2 \
 && bash $J bench cfg2lam --lam-eps 1e-9 --no-cpu-baseline \
 && bash $J bench cfg3 --config 3 --steps 5 --warmup 2 && bash $J prof cfg3 --config 3 --steps 3 --warmup 1 \
 && bash $J bench cfg3lam --config 3 --lam-eps 1e-9 --steps 2 --warmup 1 --no-cpu-baseline \
 && bash $J bench cfg4 --config 4 --steps 2 --warmup 1 \
 && bash $J bench cfg4w --config 4 --conic-variant wellcond --steps 3 --warmup 1 --no-cpu-baseline \
 && bash $J bench cfg5 --config 5 --steps 2 --warmup 1 \
 && bash $J bench cfg6 --config 6 --steps 10 --warmup 2 && bash $J prof cfg6 --config 6 --steps 5 --warmup 1
