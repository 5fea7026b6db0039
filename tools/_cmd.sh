set -e
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x -k "attention" > gpurun_out/k1.log 2>&1 || { tail -40 gpurun_out/k1.log; exit 1; }
tail -1 gpurun_out/k1.log
timeout -k 10 120 python tools/attn_bench.py --dbg --only enc,cross
timeout -k 10 120 python tools/attn_bench.py
