"""The all-layer cross K/V data gradient (c3: [15936 x 12288] . [12288 x 512] -> fp32) on split-K p4 tiles against
the default plan and an fp64 reference (tools only): relative errors and times."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    M, N, Kd = 15936, 12288, 512
    dy = (torch.randn(M, N, device="cuda", generator=g) * 0.1).bfloat16()
    w = (torch.randn(N, Kd, device="cuda", generator=g) * 0.05).bfloat16()
    ref = (dy.double() @ w.double()).float()
    out = {}
    for name, kw in (("auto", {}), ("p4 split 2", dict(kernel="p4", splitk=2)), ("p4 split 3", dict(kernel="p4", splitk=3))):   # (split p4 needs the round-4 batch-24 plan change; without it the plan takes p3)
        c = torch.empty(M, Kd, device="cuda", dtype=torch.float32)
        K.linear_dgrad(dy, w, c, **kw)
        torch.cuda.synchronize()
        err = float((c - ref).norm() / ref.norm())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            K.linear_dgrad(dy, w, c, **kw)
        e1.record()
        torch.cuda.synchronize()
        out[name] = c
        print(f"{name:12s} relerr {err:.2e}  {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us", flush=True)
        assert err < 1e-3, err


if __name__ == "__main__":
    main()
