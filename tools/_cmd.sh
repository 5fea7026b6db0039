set -e
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x -k "attention" > gpurun_out/k1.log 2>&1 || { tail -40 gpurun_out/k1.log; exit 1; }
tail -1 gpurun_out/k1.log
bash tools/gpu_suite.sh model benchq
rm -rf gpurun_out/prof
bash tools/gpu_suite.sh prof
python tools/profsum.py gpurun_out/prof/run_kernel_stats.csv 7 30
