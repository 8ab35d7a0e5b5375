# Round-4 closing run: full GPU suite, smoke, the default bench line (with its
# CPU baseline), config 6, the config-2 / config-6 kernel traces, and PMC for
# the workloads whose kernels changed last (config 2 sweeps, config 6 NLP pairs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
bash $J test && cp gpurun_out/test.log gpurun_out/test_final.log && cp gpurun_out/parity.jsonl gpurun_out/parity_final.jsonl && \
bash $J smoke && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1 && tail -1 gpurun_out/bench_final.log | tee gpurun_out/bench_final.json && \
bash $J bench cfg6 --config 6 --steps 20 --warmup 3 && \
bash $J prof cfg2 --steps 20 --warmup 3 && \
bash $J prof cfg6 --config 6 --steps 10 --warmup 2 && \
bash $J pmc cfg2 --steps 3 --warmup 1 && \
PMC_SUFFIX=@cfg6 bash $J pmc cfg6 --config 6 --steps 3 --warmup 1
