#!/bin/bash
# HBM traffic of the bench's kernels: two separate rocprofv3 --pmc passes
# (FETCH_SIZE and WRITE_SIZE cannot share a gfx950 TCC pass), no tracing
# domains combined with --pmc.  GPU box helper.
#   tools/run_pmc.sh TAG [bench.py args...]   → gpurun_out/pmc_TAG.json (merged)
set -o pipefail
tag=${1:-r01}; shift
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${tag}_$c -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_${tag}_$c.log 2>&1 \
    || { tail -20 gpurun_out/pmc_${tag}_$c.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE gpurun_out/pmc_${tag}.json
