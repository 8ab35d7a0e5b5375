set -o pipefail
mkdir -p gpurun_out
for b in 512 128 64; do
  timeout -k 10 300 python -u bench.py --config 4 --batch $b --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_b$b.log 2>&1 || exit 1
  tail -1 gpurun_out/c4_b$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('persist', $b, d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  DOPT_CONIC_SPLIT=1 timeout -k 10 300 python -u bench.py --config 4 --batch $b --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4s_b$b.log 2>&1 || exit 1
  tail -1 gpurun_out/c4s_b$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('split', $b, d['value'], d['ms_per_step'], d['roofline']['achieved'])"
done
