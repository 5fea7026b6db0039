set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread -m gpu -k "attention" > gpurun_out/k_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/k_tests.log | tail -8; [ $rc -eq 0 ] || exit 1
for v in 0 1; do ASRX_ATTN_KQ=$v timeout -k 10 120 python tools/attn_bench.py --only cross 2>&1 | grep -v amdgpu.ids; done
bash tools/ab_env.sh 2 ASRX_ATTN_KQ=0 ASRX_ATTN_KQ=1
