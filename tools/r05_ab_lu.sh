# LU iteration: QP/NLP parity subset, then A/B of VARIANTS on config 2
set -o pipefail
cd $GRAFT_REPO_ROOT
TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py tests/test_multi_rhs_gpu.py" bash tools/gpu_job.sh test && \
bash tools/ab_job.sh "$@"
