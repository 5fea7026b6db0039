"""Do the decoder's latency-bound launches overlap usefully as two half batches on two streams?  (tools only)

The c3 decoder layers' forward (12 layers, training mode, dropout 0.1, B = 64, L = 64 over T' = 249 encoder frames)
as one chain, against two B = 32 chains issued on two streams layer by layer, against the two halves one after the
other on one stream; each variant captured as a HIP graph and replayed.  Prints ms per full batch.

    python tools/dec_dualmb_probe.py [--reps 10]
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
    args = ap.parse_args()
    import asrx
    from asrx import blocks as Bk
    from asrx import kernels as K
    from asrx.functions import make_ctx, _kv_block
    cfg = CONFIGS["c3"]["cfg"]
    m = asrx.Transformer(cfg.vocab_size, cfg.input_dim, cfg.d_model, cfg.dec_len, cfg.enc_len, cfg.n_enc, cfg.n_dec,
                         cfg.n_heads, cfg.ff_dim, dropout=0.1, precision="bf16")
    sd = m.state_dict()
    sd.update(det_params(cfg, 0))
    m.load_state_dict(sd)
    m = m.cuda().train()
    dec = m.decoder
    Te, L, d, H, n = 249, 64, cfg.d_model, cfg.n_heads, cfg.n_dec
    g = torch.Generator(device="cuda").manual_seed(0)
    enc = torch.randn(64 * Te, d, device="cuda", generator=g).bfloat16()
    x64 = torch.randn(64 * L, d, device="cuda", generator=g)
    valid = torch.ones(64, L, device="cuda", dtype=torch.uint8)
    layers = list(dec._layers)
    C0 = make_ctx(m, 0.1)
    Wkv, bkv, _, _ = _kv_block(C0, dec)
    kv = torch.empty(64 * Te, n * 2 * d, dtype=torch.bfloat16, device="cuda")
    K.linear(enc, Wkv, kv, bias=bkv)
    halves = [(x64[:32 * L].clone(), kv[:32 * Te], valid[:32]), (x64[32 * L:].clone(), kv[32 * Te:], valid[32:])]

    def spec_of(v):
        return K.MaskSpec(1, True, v, v, v.stride(0))

    def chain_layer(C, x, l, kvb, v, B):
        return Bk.dec_layer_fwd(C, x, layers[l], B, L, H, spec_of(v), kvb[:, l * 2 * d:], n * 2 * d, Te)[0]

    main_s = torch.cuda.current_stream()
    side = [torch.cuda.Stream(), torch.cuda.Stream()]

    def full():
        C = make_ctx(m, 0.1)
        x = x64
        for l in range(n):
            x = chain_layer(C, x, l, kv, valid, 64)

    def dual():
        C = make_ctx(m, 0.1)
        for s in side:
            s.wait_stream(torch.cuda.current_stream())
        xs = [h[0] for h in halves]
        for l in range(n):
            for i, s in enumerate(side):
                with torch.cuda.stream(s):
                    xs[i] = chain_layer(C, xs[i], l, halves[i][1], halves[i][2], 32)
        for s in side:
            torch.cuda.current_stream().wait_stream(s)

    def serial():
        C = make_ctx(m, 0.1)
        for h in halves:
            x = h[0]
            for l in range(n):
                x = chain_layer(C, x, l, h[1], h[2], 32)

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
        print(f"{name:20s} {e0.elapsed_time(e1) / args.reps:8.3f} ms per B=64 decoder forward ({n} layers)", flush=True)


if __name__ == "__main__":
    main()
