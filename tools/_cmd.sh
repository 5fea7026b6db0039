set -e
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x -k "attention" > gpurun_out/k1.log 2>&1 || { tail -40 gpurun_out/k1.log; exit 1; }
tail -1 gpurun_out/k1.log
bash tools/gpu_suite.sh model
timeout -k 10 120 python tools/attn_bench.py
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])"; done
