# Round 6 final evidence at head (after the columns-in-flight tuning of the
# conic sweeps): the full GPU suite and smoke, the default bench line
# (config 2), config 5 with its kernel stats and loop occupancy, config 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
J=tools/gpu_job.sh
soft() { "$@"; rc=$?; [ $rc -le 1 ] || exit $rc; return 0; }
soft bash $J test
cp gpurun_out/test.log gpurun_out/test_closing.log
bash $J smoke \
 && bash $J bench cfg2 \
 && bash $J bench cfg5 --config 5 --steps 2 --warmup 1 \
 && bash $J prof cfg5 --config 5 --steps 2 --warmup 1 \
 && python3 tools/overlap.py gpurun_out/prof_cfg5 > gpurun_out/overlap_cfg5.txt \
 && python3 tools/pass_states.py gpurun_out/prof_cfg5 > gpurun_out/pass_states_cfg5.txt \
 && bash $J bench cfg4 --config 4 --steps 2 --warmup 1
