set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
DOPT_PSD_MFMA=1 TEST_PATHS=tests/test_conic_gpu.py bash $J test -k "split or config5 or large_psd or psd or all_cone" && cp gpurun_out/test.log gpurun_out/test_mfma.log && \
DOPT_PSD_MFMA=1 bash $J bench cfg5mf --config 5 --steps 2 --warmup 1 --no-cpu-baseline && \
DOPT_PSD_MFMA=1 bash $J prof cfg5mf --config 5 --steps 2 --warmup 1
