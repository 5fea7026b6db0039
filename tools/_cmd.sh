set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -m gpu -k "softmax or unfused" > gpurun_out/sm.log 2>&1 || { tail -30 gpurun_out/sm.log; exit 1; }
tail -1 gpurun_out/sm.log
for u in 1 2; do
  ASRX_SOFTMAX_U=$u timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
  echo "U=$u $(tail -1 gpurun_out/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["sub_rooflines"]["softmax_fwd"]; print(d["us"], d["frac"])')"
done
timeout -k 10 120 python - <<'PY'
import torch
sc = torch.randn(512, 249, 256, device="cuda").bfloat16(); pr = torch.empty_like(sc)
g = torch.cuda.CUDAGraph(); s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(3): pr.copy_(sc)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(20): pr.copy_(sc)
for _ in range(3): g.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 20
print(f"torch copy of the same score tensor: {us:.2f} us = {2 * sc.numel() * 2 / us / 1e3:.0f} GB/s")
PY
