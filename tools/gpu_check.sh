set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 3 > gpurun_out/b2.log 2>&1 || { tail -20 gpurun_out/b2.log; exit 1; }
tail -1 gpurun_out/b2.log
timeout -k 10 200 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b3.log 2>&1 || { tail -20 gpurun_out/b3.log; exit 1; }
tail -1 gpurun_out/b3.log
