"""Does running two half batches on two streams overlap usefully?  (tools only)

The c3 encoder forward (12 layers, training mode, dropout 0.1) on B = 64 as one chain, against two B = 32 chains
issued on two streams (their kernels free to run side by side), against the two halves one after the other on one
stream; each variant captured as a HIP graph and replayed.  Prints ms per full batch.

    python tools/dualmb_probe.py [--reps 10] [--bwd]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import torch  # noqa: E402

from oracle.ref_model import CONFIGS, det_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--layers", type=int, default=12)
    args = ap.parse_args()
    import asrx
    from asrx import blocks as Bk
    from asrx.functions import make_ctx
    cfg = CONFIGS["c3"]["cfg"]
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=0.1, precision="bf16")
    sd = m.state_dict()
    sd.update(det_params(cfg, 0))
    m.load_state_dict(sd)
    m = m.cuda().train()
    enc = m.encoder
    T, d, H = 249, cfg.d_model, cfg.n_heads
    g = torch.Generator(device="cuda").manual_seed(0)
    x64 = torch.randn(64 * T, d, device="cuda", generator=g)
    halves = [x64[:32 * T].clone(), x64[32 * T:].clone()]
    layers = list(enc._layers)[:args.layers]

    def chain(C, x, B):
        for layer in layers:
            x, _ = Bk.enc_layer_fwd(C, x, layer, B, T, H)
        return x

    main_s = torch.cuda.current_stream()
    side = [torch.cuda.Stream(), torch.cuda.Stream()]

    def full():
        C = make_ctx(m, 0.1)
        chain(C, x64, 64)

    def dual():
        C = make_ctx(m, 0.1)
        for i, s in enumerate(side):
            s.wait_stream(torch.cuda.current_stream())
        # interleave the two chains layer by layer so both streams have work queued at once
        xs = list(halves)
        for layer in layers:
            for i, s in enumerate(side):
                with torch.cuda.stream(s):
                    xs[i], _ = Bk.enc_layer_fwd(C, xs[i], layer, 32, T, H)
        for s in side:
            torch.cuda.current_stream().wait_stream(s)

    def serial():
        C = make_ctx(m, 0.1)
        for h in halves:
            chain(C, h, 32)

    res = {}
    for name, fn in (("full B=64", full), ("two B=32 streams", dual), ("two B=32 serial", serial)):
        fn()
        torch.cuda.synchronize()
        gph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(main_s)
        with torch.cuda.stream(s):
            with torch.cuda.graph(gph, stream=s):
                fn()
        torch.cuda.synchronize()
        gph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            gph.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / args.reps
        print(f"{name:20s} {res[name]:8.3f} ms per B=64 encoder forward ({args.layers} layers)", flush=True)


if __name__ == "__main__":
    main()
