# Round 6, flat diagonal chain: QP / NLP / multi-RHS parity, then config 2
# flat vs restaged strips on the same box, and the flat form's kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
T=${TAG:-flat}
TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py tests/test_multi_rhs_gpu.py tests/test_qp_small_gpu.py" bash $J test && \
DOPT_LFLAT=0 bash $J bench ${T}0 --no-cpu-baseline && \
bash $J bench ${T}1 --no-cpu-baseline && \
DOPT_LFLAT=0 bash $J bench ${T}0b --no-cpu-baseline && \
bash $J bench ${T}1b --no-cpu-baseline && \
bash $J prof ${T}cfg2 --steps 20 --warmup 3 && \
python3 tools/timeline.py gpurun_out/prof_${T}cfg2 > gpurun_out/timeline_${T}cfg2.txt
