# kernel trace of the drop-in latency bench: the small path's kernel time
# against its per-call wall time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_small -o run --output-format csv -- python3 -u tools/bench_dropin.py > gpurun_out/prof_small.log 2>&1
