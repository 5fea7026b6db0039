"""Per-shape in-kernel GEMM times of one c3 training step.

    rocprofv3 --kernel-trace -d gpurun_out/gt -o run --output-format csv -- python3 tools/gemm_table.py run
    python3 tools/gemm_table.py report gpurun_out/gt/run_kernel_trace.csv

`run` does 2 warmup steps and one logged step (every GEMM launch's kernel name and m, n, k recorded in order, no
timing events); `report` matches the logged launches with the profiler's GEMM dispatches of that last step.
For grouped launches `k` holds the summed m*n*k of the group.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOG = os.path.join(REPO, "gpurun_out", "gemm_log.json")


def run():
    sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
    sys.path.insert(0, REPO)
    import torch
    import asrx
    from asrx import kernels as K
    from asrx.train import Trainer
    from oracle.ref_model import CONFIGS, synthetic_batch
    spec = CONFIGS["c3"]
    cfg = spec["cfg"]
    torch.manual_seed(0)
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=cfg.dropout, precision="bf16").cuda().train()
    tr = Trainer(m)
    s, t, mk = synthetic_batch(cfg, spec["batch"], spec["frames"], spec["text_len"] + 1, seed=1234)
    s, t, mk = s.cuda(), t.cuda(), mk.cuda()
    for _ in range(2):
        tr.step(s, t, mk)
    torch.cuda.synchronize()
    log = []
    K.PROBE = K.KernelProbe(target="__none__", log=log)
    K.PROBE.active = True
    tr.step(s, t, mk)
    torch.cuda.synchronize()
    K.PROBE = None
    os.makedirs(os.path.dirname(LOG), exist_ok=True)
    json.dump(log, open(LOG, "w"))


def report(trace):
    import csv
    import collections
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pmc_traffic import short
    log = json.load(open(LOG))
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    names = [short(r["Kernel_Name"]) for r in rows]
    adam = [i for i, n in enumerate(names) if n.startswith("adam")]
    lo = adam[-2] + 1 if len(adam) >= 2 else 0
    gem = [(names[i], (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3)
           for i in range(lo, len(rows)) if names[i].startswith("gemm_")]
    if len(gem) != len(log):
        print(f"warning: {len(gem)} GEMM dispatches in the last step vs {len(log)} logged launches")
    agg = collections.OrderedDict()
    j, prev = 0, None
    for kn, us in gem:   # a launch split into several dispatches adds them to its logged entry
        if j < len(log) and log[j][0] == kn:
            key = tuple(log[j])
            j += 1
            a = agg.setdefault(key, [0, 0.0])
            a[0] += 1
        elif prev is not None and prev[0] == kn:
            key = prev
            a = agg[key]
        else:
            key = (kn, 0, 0, 0, 1, 1)   # not logged (e.g. the conv2 weight-gradient GEMM)
            a = agg.setdefault(key, [0, 0.0])
            a[0] += 1
        a[1] += us
        prev = key
    if j != len(log):
        print(f"warning: {len(log) - j} logged launches unmatched")
    tot = sum(v[1] for v in agg.values())
    print(f"{'us/call':>8s} {'calls':>5s} {'ms':>7s} {'TF':>6s}  m x n x k (batch, splitk)  kernel")
    for (ln, m, n, k, batch, sk), (cnt, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        fl = 2.0 * (m * n * k if n else k) * batch
        print(f"{us / cnt:8.1f} {cnt:5d} {us / 1e3:7.3f} {fl / (us / cnt) / 1e6:6.0f}  {m}x{n}x{k} ({batch},{sk})  {ln}")
    print(f"GEMM dispatches {len(gem)}, logged launches {len(log)}")
    print(f"GEMM total {tot / 1e3:.3f} ms/step")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2])
