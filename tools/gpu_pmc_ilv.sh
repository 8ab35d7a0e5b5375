#!/bin/bash
# HBM traffic of the solve kernel with and without the interleaved dispatch order
set -o pipefail
mkdir -p gpurun_out
DOPT_SOLVE_ILV=1 bash tools/run_pmc.sh r01j_ilv1 || exit 1
DOPT_SOLVE_ILV=0 bash tools/run_pmc.sh r01j_ilv0 || exit 1
