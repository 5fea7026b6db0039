"""Which host calls issue device copies (hipMemcpyAsync -> rocclr copyBuffer) in the c3 training step:
torch.profiler over one step, copy-like ops grouped by Python stack.

    python tools/copy_trace.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    import asrx
    from asrx.train import Trainer
    from oracle.ref_model import CONFIGS, synthetic_batch
    spec = CONFIGS["c3"]
    cfg = spec["cfg"]
    torch.manual_seed(0)
    model = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc,
                             cfg.n_dec, cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout, precision="bf16").cuda().train()
    tr = Trainer(model)
    s, t, m = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=1)
    s, t, m = s.cuda(), t.cuda(), m.cuda()
    for _ in range(2):
        tr.step(s, t, m)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.step(s, t, m)
        torch.cuda.synchronize()
    names = ("aten::copy_", "aten::clone", "aten::_to_copy", "aten::to", "aten::contiguous", "aten::zero_",
             "aten::fill_", "aten::cat", "aten::index", "aten::where")
    rows = [e for e in prof.key_averages(group_by_stack_n=6) if e.key in names]
    rows.sort(key=lambda e: -e.count)
    for e in rows[:30]:
        print(f"{e.count:4d}x {e.key:16s} cuda {e.device_time_total / max(1, e.count):8.1f}us")
        for fr in e.stack[:6]:
            print("        ", fr)
    kn = {}
    for e in prof.events():
        if e.device_type == torch.autograd.DeviceType.CUDA and ("opy" in e.name or "emcpy" in e.name):
            kn[e.name] = kn.get(e.name, 0) + 1
    print("device copy events:", kn)


if __name__ == "__main__":
    main()
