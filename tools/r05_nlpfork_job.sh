# NLP deferred LU on the crit stream (sides overlap it): the NLP GPU tests, an
# A/B of config 6 (fused, separate) against the HEAD build, a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_nlp_gpu.py \
  > gpurun_out/fork_tests.log 2>&1 || { tail -30 gpurun_out/fork_tests.log; exit 1; }
tail -1 gpurun_out/fork_tests.log
TAG=fork6 VARIANTS="prev base" ROUNDS=3 bash tools/ab_job.sh --config 6 --steps 10 --warmup 2 \
 && TAG=fork6sep VARIANTS="prev base" ROUNDS=2 bash tools/ab_job.sh --config 6 --nlp-separate --steps 10 --warmup 2 \
 && bash tools/gpu_job.sh prof cfg6 --config 6 --steps 5 --warmup 1 \
 && python3 tools/timeline.py gpurun_out/prof_cfg6 nlp_red_prep 2 > gpurun_out/timeline_cfg6.txt
