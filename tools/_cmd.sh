set -e
timeout -k 10 600 python -m pytest tests/test_gpu_dist.py -q -m gpu -x > gpurun_out/k1.log 2>&1 || { tail -40 gpurun_out/k1.log; exit 1; }
tail -1 gpurun_out/k1.log
bash tools/gpu_suite.sh model benchq
