set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread -m gpu -k "attention or dropgen or softmax or ewise or ws" > gpurun_out/k_tests.log 2>&1; rc=$?; echo "kernel tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/k_tests.log | tail -15; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/blas_ref.py --only "dec ffn1 dg512,dec qkv dg512,dec out dg512,dec ffn2 fwd res" --variants p3,ring,ws64 --noblas --nogrouped 2>&1 | grep -v amdgpu.ids
bash tools/ab_env.sh 2 ASRX_WS64=0 ASRX_WS64=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_train_parity.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -m gpu -k "g64l or c5 or long or submodule or standalone or bench_batch" > gpurun_out/long_tests.log 2>&1; rc=$?; echo "model tests rc=$rc"; tail -4 gpurun_out/long_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/attn_bench.py --only enc,cross,cross24k,dec 2>&1 | grep -v amdgpu.ids
