# Round 6 closing evidence at head: the full GPU suite and smoke, the default
# bench line (config 2, with its CPU baseline), the conic configs 4 / 5 after
# the non-temporal A_moi loads (bench lines, config-5 kernel stats and loop
# occupancy, PMC traffic of both LSQR kernels).  A failing test (exit 1) does
# not stop the evidence steps; a fault, abort or time limit ends the script.
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
 && bash $J pmc cfg5 --config 5 --steps 1 --warmup 1 \
 && bash $J bench cfg4 --config 4 --steps 2 --warmup 1 \
 && bash $J pmc cfg4 --config 4 --steps 1 --warmup 1 \
 && bash $J bench cfg4w --config 4 --conic-variant wellcond --steps 3 --warmup 1 --no-cpu-baseline
