"""Cold/warm HBM fraction of the unfused-path softmax kernels (bench.sub_rooflines' measurement) for each
short-row variant (asrx_set_tuning "softmax_u" = 1, 2, 4).

    python tools/softmax_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import bench  # noqa: E402
from asrx import kernels as K  # noqa: E402

for u in (1, 2, 4):
    K.set_tuning("softmax_u", u)
    r = bench.sub_rooflines(64, 249, 512, 8, 2048, 0.1)
    print(json.dumps({"u": u, **{k: {f: r[k][f] for f in ("us", "frac", "us_warm", "frac_warm")}
                                  for k in ("softmax_fwd", "softmax_bwd", "layernorm_fwd", "layernorm_bwd")}}),
          flush=True)
K.set_tuning("softmax_u", 0)
