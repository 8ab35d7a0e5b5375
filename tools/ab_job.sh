# A/B bench of engine builds in one GPU call: VARIANTS="name ..." (default
# build = "base"), ROUNDS interleaved rounds, extra bench.py args in $@.
# → gpurun_out/ab_<tag>.txt (solves/s and the phase breakdown per run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/ab_${TAG:-ab}.txt
: > $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then lib=""; else lib=diffopt.jl_amd/diffopt_amd/variants/libdiffopt_$v.so; fi
    DOPT_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab_run.log').read().strip().splitlines()[-1])
ro=d.get('roofline',{}); ph=ro.get('phases_ms_per_step',{}); ph['lu_live']=ro.get('avg_launch_ms',0)
print('$v', 'round $r', round(d['value']), 'ms/step %.4f' % d['ms_per_step'], ' '.join('%s=%.4f' % (k, v) for k, v in ph.items()))
" | tee -a $out
  done
done
