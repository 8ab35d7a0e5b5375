# Round-5 refresh after the speculative NLP LU launch: full GPU suite, smoke,
# config 6 fused / separate bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_r05final.log \
 && bash $J smoke \
 && bash $J bench cfg6 --config 6 --steps 10 --warmup 2 \
 && bash $J bench cfg6sep --config 6 --nlp-separate --steps 10 --warmup 2 --no-cpu-baseline
