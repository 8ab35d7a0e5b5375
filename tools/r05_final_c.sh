# Round-5 closing refresh, part C: conic configs 4 / 5, NLP config 6 (+ trace),
# drop-in latency
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J bench cfg4 --config 4 --steps 2 --warmup 1 \
 && bash $J bench cfg4w --config 4 --conic-variant wellcond --steps 3 --warmup 1 --no-cpu-baseline \
 && bash $J bench cfg5 --config 5 --steps 2 --warmup 1 \
 && bash $J bench cfg6 --config 6 --steps 10 --warmup 2 \
 && bash $J prof cfg6 --config 6 --steps 5 --warmup 1 \
 && PMC_SUFFIX=@cfg6 bash $J pmc cfg6 --config 6 --steps 3 --warmup 1 \
 && timeout -k 10 300 python3 -u tools/bench_dropin.py > gpurun_out/dropin.jsonl 2>gpurun_out/dropin.err
