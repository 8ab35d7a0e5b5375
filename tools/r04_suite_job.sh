set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_full.log && cp gpurun_out/parity.jsonl gpurun_out/parity_full.jsonl && \
bash $J bench cfg2 --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
DOPT_SPLIT_NC=4 bash $J bench cfg5nc4 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J prof cfg5 --config 5 --steps 2 --warmup 1 && \
bash $J prof cfg2 --steps 20 --warmup 3
