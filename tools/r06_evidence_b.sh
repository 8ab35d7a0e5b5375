# Round 6 evidence, part B: the conic configs 4 / 5 (kernel stats, the config-5
# iteration-loop occupancy, PMC at head: VERDICT r05 weak 2) and the sparse
# route's PMC (configs 7 / 8)
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J bench cfg5 --config 5 --steps 2 --warmup 1 \
 && bash $J prof cfg5 --config 5 --steps 2 --warmup 1 \
 && python3 tools/overlap.py gpurun_out/prof_cfg5 > gpurun_out/overlap_cfg5.txt \
 && bash $J pmc cfg5 --config 5 --steps 1 --warmup 1 \
 && bash $J bench cfg4 --config 4 --steps 2 --warmup 1 \
 && bash $J pmc cfg4 --config 4 --steps 1 --warmup 1 \
 && bash $J bench cfg4w --config 4 --conic-variant wellcond --steps 3 --warmup 1 --no-cpu-baseline \
 && PMC_SUFFIX=@cfg7 bash $J pmc cfg7 --config 7 --steps 2 --warmup 1 \
 && PMC_SUFFIX=@cfg8 bash $J pmc cfg8 --config 8 --steps 2 --warmup 1
