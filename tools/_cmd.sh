set -e
timeout -k 10 300 python tools/gemm_bench.py --variants auto,p3,reg > gpurun_out/gemm_ab.log 2>&1
cat gpurun_out/gemm_ab.log
rm -rf gpurun_out/prof gpurun_out/pmcf gpurun_out/pmcw
bash tools/gpu_suite.sh prof pmcf pmcw bench
