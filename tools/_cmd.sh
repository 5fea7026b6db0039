set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -m gpu -k "softmax or unfused" > gpurun_out/sm.log 2>&1 || { tail -30 gpurun_out/sm.log; exit 1; }
tail -1 gpurun_out/sm.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python3 -c 'import json,sys; D=json.loads(sys.stdin.read()); print(D["ms_per_step"], {k: (v["us"], v["frac"]) for k, v in D["sub_rooflines"].items()})'
