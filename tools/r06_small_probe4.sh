#!/bin/bash
# small-path LU A/B (probe only): head vs U rows on two waves (w2), twice each
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/small_p4.txt
for r in 1 2; do
  for v in blk w2 blk_st w2_st; do
    echo "== $v ($r)" >> gpurun_out/small_p4.txt
    timeout -k 10 60 tools/probebin_blk/small_probe_$v >> gpurun_out/small_p4.txt 2>&1 || exit 1
  done
done
for shp in "20 30 10" "40 100 20" "60 70 40" "64 64 0" "3 2 1"; do
  for v in blk w2; do
    echo "== $v $shp" >> gpurun_out/small_p4.txt
    timeout -k 10 60 tools/probebin_blk/small_probe_$v $shp >> gpurun_out/small_p4.txt 2>&1 || exit 1
  done
done
grep -E "==|kernel|LU |diff" gpurun_out/small_p4.txt
