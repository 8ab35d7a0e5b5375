# Round-5 closing check at head: full GPU suite, smoke, the default bench line
# (config 2) and config 6, drop-in latency
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_r05final.log \
 && bash $J smoke \
 && bash $J bench cfg2 \
 && bash $J bench cfg6 --config 6 --steps 10 --warmup 2 \
 && timeout -k 10 300 python3 -u tools/bench_dropin.py > gpurun_out/dropin.jsonl 2>gpurun_out/dropin.err
