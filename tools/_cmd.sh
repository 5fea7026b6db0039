set -e
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x -k "grouped" > gpurun_out/k1.log 2>&1 || { tail -40 gpurun_out/k1.log; exit 1; }
tail -1 gpurun_out/k1.log
for v in "ASRX_GROUPED_XCD=0" "ASRX_GROUPED_XCD=1"; do
  for i in 1 2; do env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['achieved'])"; done
done
