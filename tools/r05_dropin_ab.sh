# drop-in latency: HEAD build, this build, and VARIANT (one round each, twice)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
  for v in prev base ${VARIANT}; do
    lib=""; [ "$v" != base ] && lib=diffopt.jl_amd/diffopt_amd/variants/libdiffopt_$v.so
    DOPT_LIB=$lib timeout -k 10 300 python3 -u tools/bench_dropin.py > gpurun_out/dropin_${v}_$r.jsonl 2>/dev/null || exit 1
  done
done
