#!/bin/bash
# One parameterised runner for the GPU box (gpurun).  Every GPU step runs under
# its own time limit; the first failure ends the script.
#
#   tools/gpu_job.sh test  [pytest args]          -m gpu parity suite (TEST_PATHS, default tests) → gpurun_out/test.log
#   tools/gpu_job.sh smoke                        __graft_entry__.smoke()
#   tools/gpu_job.sh bench TAG [bench.py args]    one bench line → gpurun_out/bench_TAG.json
#   tools/gpu_job.sh prof  TAG [bench.py args]    rocprofv3 --kernel-trace --stats → gpurun_out/prof_TAG/
#   tools/gpu_job.sh pmc   TAG [bench.py args]    FETCH_SIZE and WRITE_SIZE, one pass each
#                                                 → gpurun_out/pmc_TAG.json (tools/pmc_summary.py)
# Steps can be chained in one gpurun call with &&.  Environment overrides
# (e.g. DOPT_LU=0) are passed through.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
mode=$1; shift
case "$mode" in
  test)
    export DOPT_PARITY_LOG=gpurun_out/parity.jsonl
    rm -f $DOPT_PARITY_LOG
    timeout -k 10 900 python -u -m pytest ${TEST_PATHS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
      > gpurun_out/test.log 2>&1
    rc=$?; tail -5 gpurun_out/test.log; exit $rc ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; tail -3 gpurun_out/smoke.log; exit $rc ;;
  bench)
    tag=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$tag.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_$tag.log | tee gpurun_out/bench_$tag.json; exit $rc ;;
  prof)
    tag=$1; shift
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$tag.log 2>&1
    rc=$?; tail -1 gpurun_out/prof_$tag.log
    [ $rc -eq 0 ] && python3 tools/kstats.py gpurun_out/prof_$tag
    exit $rc ;;
  pmc)
    tag=$1; shift
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${tag}_$c -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/pmc_${tag}_$c.log 2>&1 \
        || { tail -20 gpurun_out/pmc_${tag}_$c.log; exit 1; }
    done
    python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE \
      gpurun_out/pmc_${tag}.json ${PMC_SUFFIX:-} ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
