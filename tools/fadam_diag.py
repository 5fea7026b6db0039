"""Which parameters differ between the fused-AdamW and the separate-AdamW Trainer after 2 steps (diagnostic)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from test_gpu_fused_adam import run  # noqa: E402

ref, l0 = run("c3", False, False, 2, 2)
tr, l1 = run("c3", True, False, 2, 2)
print("losses", l0, l1, "cover ranges", len(tr._cover or []))
st = tr.store
names = {id(p): n for n, p in tr.model.named_parameters()}
bad = 0
for p_ref, p in zip(ref.store.params, st.params):
    o, k = st.offset(p), p.numel()
    for nm, a, b in (("p", ref.store.flat, st.flat), ("m", ref.m, tr.m), ("v", ref.v, tr.v),
                     ("g", ref.store.grad, st.grad)):
        d = (a[o:o + k] - b[o:o + k]).abs().max().item()
        if d != 0:
            cov = any(c0 <= o < c0 + ck for c0, ck in (tr._cover or []))
            print(f"{names.get(id(p), '?'):60s} {nm} maxdiff {d:.3e} covered {cov} off {o} n {k}")
            bad += 1
print("differing", bad)
