# config-4 persistent co-iterated LSQR vs rows per lane (DOPT_PAIR_K) and
# columns in flight (DOPT_PAIR_NC); KS / NCS lists
set -o pipefail
mkdir -p gpurun_out
for k in ${KS:-8 4}; do for nc in ${NCS:-3}; do
  make -s -C diffopt.jl_amd clean && make -s -j16 -C diffopt.jl_amd CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function -DDOPT_PAIR_K=$k -DDOPT_PAIR_NC=$nc" > /dev/null 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4pk$k.log 2>&1 || exit 1
  tail -1 gpurun_out/c4pk$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('PK', $k, 'NC', $nc, d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done; done
