# Round 5 LU iteration: QP + NLP parity tests, the config-2 kernel trace and
# per-dispatch PMC traffic (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
T=${TAG:-lu}
TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py tests/test_multi_rhs_gpu.py" bash $J test && \
bash $J prof ${T}cfg2 --steps 20 --warmup 3 && \
bash $J pmc ${T}cfg2 --steps 3 --warmup 1 && \
python3 tools/pmc_dispatch.py gpurun_out/pmc_${T}cfg2_FETCH_SIZE gpurun_out/pmc_${T}cfg2_WRITE_SIZE > gpurun_out/pmcd_${T}cfg2.txt
