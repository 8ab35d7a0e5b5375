# SQ counters (one pass) of the config-6 step: what paces the NLP reduction kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
timeout -s KILL 180 rocprofv3 --pmc $SQ -d gpurun_out/sq_cfg6 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config 6 --steps 3 --warmup 1 > gpurun_out/sq_cfg6.log 2>&1
