#!/bin/bash
# conic bench line(s) on the GPU box: tools/gpu_conic.sh TAG [bench args...]
set -o pipefail
tag=$1; shift
timeout -k 10 400 python bench.py "$@" > gpurun_out/bc_$tag.log 2>&1 || { tail -20 gpurun_out/bc_$tag.log; exit 1; }
tail -1 gpurun_out/bc_$tag.log
