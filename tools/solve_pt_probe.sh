# config-2 step time vs the blocked solves' workgroup size (DOPT_SOLVE_PT)
set -o pipefail
mkdir -p gpurun_out
for pt in ${PTS:-512 256}; do
  make -s -C diffopt.jl_amd clean && make -s -j16 -C diffopt.jl_amd CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function -DDOPT_SOLVE_PT=$pt" > /dev/null 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline ${ARGS:-} > gpurun_out/spt$pt.log 2>&1 || exit 1
  tail -1 gpurun_out/spt$pt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('PT', $pt, d['value'], d['ms_per_step'], d['roofline']['phases_ms_per_step'])"
done
