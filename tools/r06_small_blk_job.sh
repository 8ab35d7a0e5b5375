#!/bin/bash
# small-path LU: the 16-block MFMA form (blk: blocked U sweep; steps: the
# step-by-step U sweep) against the rank-4 groups (grp) — probe at the config-1
# shape and ragged shapes, thread-0 stamps
set -o pipefail
mkdir -p gpurun_out
for v in blk steps grp blk_st steps_st grp_st; do
  echo "== $v" >> gpurun_out/small_blk.txt
  timeout -k 10 60 tools/probebin_blk/small_probe_$v >> gpurun_out/small_blk.txt 2>&1 || exit 1
done
for shp in "20 30 10" "40 100 20" "60 70 40" "30 200 0" "100 40 27" "3 2 1"; do
  echo "== blk $shp" >> gpurun_out/small_blk.txt
  timeout -k 10 60 tools/probebin_blk/small_probe_blk $shp >> gpurun_out/small_blk.txt 2>&1 || exit 1
done
cat gpurun_out/small_blk.txt
