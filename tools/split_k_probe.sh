# split LSQR throughput vs rows per split row block (DOPT_SPLIT_K); CFG=4 or 5
set -o pipefail
mkdir -p gpurun_out
for k in ${KS:-1 2 4}; do
  make -s -C diffopt.jl_amd clean && make -s -j16 -C diffopt.jl_amd CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function -DDOPT_SPLIT_K=$k" > /dev/null 2>&1 || exit 1
  DOPT_CONIC_SPLIT=1 timeout -k 10 300 python -u bench.py --config ${CFG:-4} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c${CFG:-4}k$k.log 2>&1 || exit 1
  tail -1 gpurun_out/c${CFG:-4}k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('splitK', $k, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline'].get('lsqr_iterations_mean'))"
done
