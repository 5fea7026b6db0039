set -e
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x -k "grouped" > gpurun_out/k1.log 2>&1 || { tail -40 gpurun_out/k1.log; exit 1; }
tail -1 gpurun_out/k1.log
bash tools/gpu_suite.sh model
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['achieved'])"; done
export TMPDIR=/tmp
rm -rf gpurun_out/gt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gt -o run --output-format csv -- python3 tools/gemm_table.py run > /dev/null 2>&1
python3 tools/gemm_table.py report gpurun_out/gt/run_kernel_trace.csv | head -8
