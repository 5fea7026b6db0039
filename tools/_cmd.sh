set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train_parity.py -q --timeout 300 --timeout-method thread -m gpu -k "ws or gemm or bench_batch" > gpurun_out/k_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/k_tests.log | tail -8; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh 3 ASRX_WS_QKV=0 ASRX_WS_QKV=1
