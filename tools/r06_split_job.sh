# Round 6: the small-path probe inlined / out of line, the
# sparse route's, plug point's and QP tests (incl. the weakly-active rows),
# QP / NLP parity under the split column schedule (DOPT_LSPLIT), then config 2
# in all four flat / split combinations (two rounds) and the split kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
J=tools/gpu_job.sh
mkdir -p gpurun_out
for v in inl noinl r05_inl r05_noinl; do
  timeout -k 10 60 tools/probebin_r06/small_probe_$v > gpurun_out/probe_$v.txt 2>&1 || exit 1
done
TEST_PATHS="tests/test_sparse_gpu.py tests/test_lhs_solve_gpu.py tests/test_qp_gpu.py tests/test_qp_small_gpu.py tests/test_nlp_gpu.py" bash $J test && cp gpurun_out/test.log gpurun_out/test_a.log && \
DOPT_LSPLIT=1 TEST_PATHS="tests/test_qp_gpu.py tests/test_nlp_gpu.py tests/test_multi_rhs_gpu.py" bash $J test || exit 1
for r in a b; do
 DOPT_LFLAT=0 DOPT_LSPLIT=0 bash $J bench f0s0$r --no-cpu-baseline && \
 DOPT_LFLAT=1 DOPT_LSPLIT=0 bash $J bench f1s0$r --no-cpu-baseline && \
 DOPT_LFLAT=0 DOPT_LSPLIT=1 bash $J bench f0s1$r --no-cpu-baseline && \
 DOPT_LFLAT=1 DOPT_LSPLIT=1 bash $J bench f1s1$r --no-cpu-baseline || exit 1
done
DOPT_LSPLIT=1 bash $J prof split --steps 20 --warmup 3 && \
python3 tools/timeline.py gpurun_out/prof_split > gpurun_out/timeline_split.txt
