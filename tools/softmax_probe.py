"""Cold/warm HBM fraction of the unfused-path softmax kernels (bench.sub_rooflines' measurement) for each
short-row variant (asrx_set_tuning "softmax_u" = 1, 2, 4) and access policy (ASRX_SOFTMAX_NT: 0 = default,
1 = non-temporal forward, 3 = non-temporal forward and backward).

    python tools/softmax_probe.py [--u 1,2,4] [--nt 0]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import bench  # noqa: E402
from asrx import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--u", default="1,2,4")
ap.add_argument("--nt", default="0")
args = ap.parse_args()
for nt in args.nt.split(","):
    os.environ["ASRX_SOFTMAX_NT"] = nt
    for u in (int(x) for x in args.u.split(",")):
        K.set_tuning("softmax_u", u)
        r = bench.sub_rooflines(64, 249, 512, 8, 2048, 0.1)
        print(json.dumps({"nt": nt, "u": u, **{k: {f: r[k][f] for f in ("us", "frac", "us_warm", "frac_warm")}
                                               for k in ("softmax_fwd", "softmax_bwd", "layernorm_fwd",
                                                         "layernorm_bwd")}}), flush=True)
K.set_tuning("softmax_u", 0)
