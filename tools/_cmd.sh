set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for rw in 1 2 4; do
  ASRX_LN_RW=$rw timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu -k "layernorm or ln_" > gpurun_out/ln.log 2>&1 || { tail -30 gpurun_out/ln.log; exit 1; }
  echo "RW=$rw $(tail -1 gpurun_out/ln.log)"
done
for rw in 1 2 4 1 2 4; do
  ASRX_LN_RW=$rw timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  echo "RW=$rw $(tail -1 gpurun_out/b.log | python3 -c 'import json,sys; D=json.loads(sys.stdin.read()); d=D["sub_rooflines"]["layernorm_fwd"]; print(D["ms_per_step"], d["us"], d["frac"])')"
done
