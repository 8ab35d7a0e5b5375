# Round-5 last check at head: full GPU suite and smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_r05final.log && bash $J smoke
