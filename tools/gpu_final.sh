#!/bin/bash
# Round artefacts (tag $1): PMC traffic (configs 2, 3) merged into
# profiles/pmc_latest.json, then bench lines (config 2 with CPU baseline,
# config 3), then the rocprofv3 kernel-trace summary of the config-2 bench.
set -o pipefail
tag=${1:-r01f}
mkdir -p gpurun_out
bash tools/run_pmc.sh ${tag}_c2 || exit 1
bash tools/run_pmc.sh ${tag}_c3 --config 3 || exit 1
python - <<PY || exit 1
import json
p = "profiles/pmc_latest.json"
d = json.load(open(p))
for t in ["${tag}_c2", "${tag}_c3"]:
    k = json.load(open(f"gpurun_out/pmc_{t}.json"))["kernels"]
    # config-3 entries keyed by config (the bench reads the key of its config)
    suffix = "" if t.endswith("c2") else "@cfg3"
    d["kernels"].update({kk + suffix: v for kk, v in k.items()})
json.dump(d, open(p, "w"), indent=1)
json.dump(d, open("gpurun_out/pmc_latest.json", "w"), indent=1)
PY
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 > gpurun_out/bench_${tag}_c2.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c2.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c2.log
timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_${tag}_c3.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_c3.log; exit 1; }
tail -1 gpurun_out/bench_${tag}_c3.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c2 -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_${tag}_c2.log 2>&1 || { tail -20 gpurun_out/prof_${tag}_c2.log; exit 1; }
tail -1 gpurun_out/prof_${tag}_c2.log
python tools/kstats.py gpurun_out/prof_${tag}_c2/run_kernel_stats.csv 23
