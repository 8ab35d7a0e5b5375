# Round-4 closing run: full GPU suite, smoke, the default bench line (with its
# CPU baseline), the config-2 kernel trace, and PMC for the workloads whose
# kernels changed this round (config 5 fused split LSQR, config 6 NLP)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_final.log && cp gpurun_out/parity.jsonl gpurun_out/parity_final.jsonl && \
bash $J smoke && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1 && tail -1 gpurun_out/bench_final.log | tee gpurun_out/bench_final.json && \
bash $J prof cfg2 --steps 20 --warmup 3 && \
bash $J bench cfg6 --config 6 --steps 20 --warmup 3 && \
bash $J prof cfg6 --config 6 --steps 10 --warmup 2 && \
bash $J pmc cfg5 --config 5 --steps 1 --warmup 1 && \
PMC_SUFFIX=@cfg6 bash $J pmc cfg6 --config 6 --steps 3 --warmup 1
