# Round-5 closing refresh, part A: full GPU suite, smoke, the config-2 headline
# line (with its CPU baseline), its kernel trace + step timeline, its PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_r05final.log \
 && bash $J smoke \
 && bash $J bench cfg2 \
 && bash $J prof cfg2 --steps 20 --warmup 3 \
 && python3 tools/timeline.py gpurun_out/prof_cfg2 > gpurun_out/timeline_cfg2.txt \
 && bash $J pmc cfg2 --steps 5 --warmup 2
