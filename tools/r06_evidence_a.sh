# Round 6 evidence, part A: the small path's blocked LU (probe, tests, drop-in
# latency), the changed QP / NLP paths' GPU tests, then configs 2, 3,
# 2 (--lam-eps) and 6 at head, each with its PMC traffic (the stale `traffic`
# fields of VERDICT r05 weak 10).  A failing test (exit 1) does not stop the
# evidence steps; a fault, abort or time limit (any other non-zero status)
# ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
soft() { "$@"; rc=$?; [ $rc -le 1 ] || exit $rc; return 0; }
soft bash tools/r06_small_blk_job.sh
TEST_PATHS="tests/test_qp_small_gpu.py tests/test_qp_gpu.py tests/test_multi_rhs_gpu.py tests/test_nlp_gpu.py tests/test_lhs_solve_gpu.py tests/test_params_gpu.py tests/test_model_api_gpu.py" soft bash $J test
cp gpurun_out/test.log gpurun_out/test_uinv.log
soft timeout -k 10 300 python3 -u tools/bench_dropin.py > gpurun_out/dropin.jsonl 2>gpurun_out/dropin.err
bash $J bench cfg2 --no-cpu-baseline \
 && bash $J prof cfg2 --steps 20 --warmup 3 \
 && python3 tools/timeline.py gpurun_out/prof_cfg2 > gpurun_out/timeline_cfg2.txt \
 && bash $J bench cfg3 --config 3 --steps 5 --warmup 2 \
 && PMC_SUFFIX=@cfg3 bash $J pmc cfg3 --config 3 --steps 2 --warmup 1 \
 && bash $J prof cfg3 --config 3 --steps 3 --warmup 1 \
 && bash $J bench cfg2lam --lam-eps 1e-9 --no-cpu-baseline \
 && PMC_SUFFIX=@lam bash $J pmc cfg2lam --lam-eps 1e-9 --steps 3 --warmup 1 \
 && bash $J bench cfg6 --config 6 --steps 10 --warmup 2 \
 && PMC_SUFFIX=@cfg6 bash $J pmc cfg6 --config 6 --steps 3 --warmup 1 \
 && bash $J pmc cfg2 --steps 5 --warmup 2
