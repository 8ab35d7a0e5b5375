# SQ counters (one pass, 8 SQ counters) of the config-2 and config-3 steps → gpurun_out/sq_cfg{2,3}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
timeout -s KILL 180 rocprofv3 --pmc $SQ -d gpurun_out/sq_cfg2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/sq_cfg2.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $SQ -d gpurun_out/sq_cfg3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 3 --steps 2 --warmup 1 > gpurun_out/sq_cfg3.log 2>&1
