"""LayerNorm forward/backward micro-benchmark on the c3 encoder shape (15936 x 512): time per call and achieved HBM
GB/s (algorithmic bytes: every operand read once, every output written once), cold (rotating buffer sets larger
than the 256 MiB Infinity Cache, as bench.py's sub_rooflines) and warm (one set), for every kernel variant.

    python tools/ln_bench.py [--pf 8,1,2,4] [--bpc 2,4,8] [--blocks 512,1024,2048]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from asrx import kernels as K  # noqa: E402
from bench import COLD_BYTES, _graph_time_ms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pf", default="8,1,2,4")
    ap.add_argument("--bpc", default="2,4,8")
    ap.add_argument("--blocks", default="512,1024,2048")
    ap.add_argument("--rows", type=int, default=64 * 249)
    args = ap.parse_args()
    d, rows = 512, args.rows
    g = torch.Generator(device="cuda").manual_seed(0)
    gamma = torch.rand(d, device="cuda", generator=g) + 0.5
    beta = torch.randn(d, device="cuda", generator=g)
    fby = rows * d * (4 + 2) + rows * 8
    bby = rows * d * (4 + 2 + 4 + 4 + 2) + rows * 8
    nf = max(2, -(-COLD_BYTES // fby))
    nb = max(2, -(-COLD_BYTES // bby))
    fsets = [(torch.randn(rows, d, device="cuda", generator=g),
              torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)) for _ in range(nf)]
    fst = [K.layernorm_fwd(x, gamma, beta, y) for x, y in fsets]
    ffns = [lambda x=x, y=y: K.layernorm_fwd(x, gamma, beta, y) for x, y in fsets]
    for pf in [int(v) for v in args.pf.split(",")]:
        K.set_tuning("ln_pf", pf)
        for bpc in ([int(v) for v in args.bpc.split(",")] if pf != 8 else [0]):
            K.set_tuning("ln_bpc", bpc)
            tc, tw = _graph_time_ms(ffns) * 1e-3, _graph_time_ms(ffns[:1]) * 1e-3
            print(f"ln_fwd rows={rows} pf={pf} bpc={bpc}: cold {tc*1e6:6.2f} us {fby/tc/1e9:5.0f} GB/s "
                  f"({fby/tc/8e12:.3f}) | warm {tw*1e6:6.2f} us {fby/tw/1e9:5.0f} GB/s", flush=True)
    K.set_tuning("ln_bpc", 0)
    # floor: the same bytes moved by a plain fp32 -> bf16 cast (torch's elementwise kernel), and by asrx_cast
    cfns = [lambda x=x, y=y: y.copy_(x) for x, y in fsets]
    tc, tw = _graph_time_ms(cfns) * 1e-3, _graph_time_ms(cfns[:1]) * 1e-3
    print(f"floor torch cast fp32->bf16 same bytes: cold {tc*1e6:6.2f} us {fby/tc/1e9:5.0f} GB/s ({fby/tc/8e12:.3f}) | "
          f"warm {tw*1e6:6.2f} us", flush=True)
    big = [(torch.randn(rows * 8, d, device="cuda", generator=g), torch.empty(rows * 8, d, device="cuda",
                                                                          dtype=torch.bfloat16)) for _ in range(2)]
    bfl = [lambda x=x, y=y: y.copy_(x) for x, y in big]
    tc = _graph_time_ms(bfl, launches=4) * 1e-3
    print(f"floor torch cast, 8x the rows: {tc*1e6:6.2f} us {8*fby/tc/1e9:5.0f} GB/s ({8*fby/tc/8e12:.3f})", flush=True)
    del big, bfl
    bsets = []
    for i in range(nb):
        x, _ = fsets[i % nf]
        mean, rstd = fst[i % nf]
        bsets.append((x, torch.randn(rows, d, device="cuda", generator=g).bfloat16(), mean, rstd,
                      torch.randn(rows, d, device="cuda", generator=g),
                      torch.empty(rows, d, device="cuda", dtype=torch.bfloat16)))
    dgb = torch.zeros(2 * d, device="cuda")
    bfns = [lambda s=s: K.layernorm_bwd(s[0], s[1], gamma, s[2], s[3], dgb, dres=s[4], dx_drop=s[5], dropout_p=0.1,
                                         seed=3, defer=[]) for s in bsets]
    for pf in [int(v) for v in args.pf.split(",")]:
        K.set_tuning("ln_pf", pf)
        for blocks in [int(v) for v in args.blocks.split(",")]:
            K.LN_BWD_BLOCKS = blocks
            tc, tw = _graph_time_ms(bfns) * 1e-3, _graph_time_ms(bfns[:1]) * 1e-3
            print(f"ln_bwd rows={rows} pf={pf} blocks={blocks}: cold {tc*1e6:6.2f} us {bby/tc/1e9:5.0f} GB/s "
                  f"({bby/tc/8e12:.3f}) | warm {tw*1e6:6.2f} us {bby/tw/1e9:5.0f} GB/s", flush=True)
    K.set_tuning("ln_pf", 0)


if __name__ == "__main__":
    main()
