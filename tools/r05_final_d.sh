# Round-5 closing refresh after the host-flow changes (side read-backs, the
# deferred NLP factor, the plug point's factor reuse): full GPU suite, smoke,
# the config-2 line + trace + timeline, config 6 (fused, separate) + trace,
# config 5, drop-in latency
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_r05final.log \
 && bash $J smoke \
 && bash $J bench cfg2 \
 && bash $J prof cfg2 --steps 20 --warmup 3 \
 && python3 tools/timeline.py gpurun_out/prof_cfg2 > gpurun_out/timeline_cfg2.txt \
 && bash $J bench cfg6 --config 6 --steps 10 --warmup 2 \
 && bash $J bench cfg6sep --config 6 --nlp-separate --steps 10 --warmup 2 --no-cpu-baseline \
 && bash $J prof cfg6 --config 6 --steps 5 --warmup 1 \
 && python3 tools/timeline.py gpurun_out/prof_cfg6 nlp_red_prep 2 > gpurun_out/timeline_cfg6.txt \
 && bash $J bench cfg5 --config 5 --steps 2 --warmup 1 \
 && timeout -k 10 300 python3 -u tools/bench_dropin.py > gpurun_out/dropin.jsonl 2>gpurun_out/dropin.err
