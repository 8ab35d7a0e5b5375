set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
DOPT_PARITY_CALIBRATE=1 TEST_PATHS=tests/test_conic_gpu.py bash $J test && cp gpurun_out/test.log gpurun_out/test_fused.log && cp gpurun_out/parity.jsonl gpurun_out/parity_fused.jsonl && \
bash $J bench cfg2 --steps 20 --warmup 3 --no-cpu-baseline && \
DOPT_SYM_TPB=256 bash $J bench cfg2tpb --steps 20 --warmup 3 --no-cpu-baseline && \
bash $J bench cfg5 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
DOPT_SPLIT_FUSE=0 bash $J bench cfg5nofuse --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
DOPT_SPLIT_NW=8 bash $J bench cfg5nw8 --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
bash $J prof cfg5 --config 5 --steps 2 --warmup 1 && \
DOPT_PARITY_CALIBRATE=1 DOPT_SPLIT_FUSE=0 TEST_PATHS=tests/test_conic_gpu.py bash $J test -k "split or config5 or large_psd" && cp gpurun_out/test.log gpurun_out/test_nofuse.log && \
DOPT_LFLOW=1 timeout -k 10 180 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_cfg2flow.log 2>&1 && tail -1 gpurun_out/bench_cfg2flow.log && \
DOPT_LFLOW=1 TEST_PATHS=tests/test_qp_gpu.py bash $J test && cp gpurun_out/test.log gpurun_out/test_flow.log
