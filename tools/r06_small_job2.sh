#!/bin/bash
# small path: LU variant probes, then the drop-in latency under rocprofv3
# (kernel durations of the QPModel sequence)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/r06_small_blk_job.sh > /dev/null \
 && timeout -k 10 300 python3 -u tools/bench_dropin.py --reps 30 > gpurun_out/dropin2.jsonl 2>gpurun_out/dropin2.err \
 && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_dropin -o run --output-format csv \
      -- python3 tools/bench_dropin.py --reps 30 > gpurun_out/prof_dropin.log 2>&1 \
 && python3 tools/kstats.py gpurun_out/prof_dropin > gpurun_out/dropin_kstats.txt
cat gpurun_out/small_blk.txt | grep -E "==|kernel|LU|cycles|diff" | head -120
