#!/bin/bash
# small-path blocked LU variants (probe): blk (IEEE division, branch), rcp
# (v_rcp + Newton, branch-free panel), t2 (two trailing tiles per wave at a
# time), rcpt2 (both) — config-1 shape timings, thread-0 stamps, ragged shapes
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/small_blk.txt
for v in blk rcp t2 rcpt2 blk_st rcp_st t2_st rcpt2_st; do
  echo "== $v" >> gpurun_out/small_blk.txt
  timeout -k 10 60 tools/probebin_blk/small_probe_$v >> gpurun_out/small_blk.txt 2>&1 || exit 1
done
for v in blk rcpt2; do
  for shp in "20 30 10" "40 100 20" "60 70 40" "30 200 0" "100 40 27" "3 2 1" "1 1 0" "16 0 0" "64 64 0"; do
    echo "== $v $shp" >> gpurun_out/small_blk.txt
    timeout -k 10 60 tools/probebin_blk/small_probe_$v $shp >> gpurun_out/small_blk.txt 2>&1 || exit 1
  done
done
cat gpurun_out/small_blk.txt
