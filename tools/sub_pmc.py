"""One pass of bench.sub_rooflines (the per-kernel cold/warm measurements at the c3 encoder shapes: unfused
softmax forward/backward, LayerNorm forward/backward, Q/K/V projection, attention forward) — the program the
PMC passes run, so the softmax and LayerNorm kernels get HBM counters of their own (they are not, or not alone,
in the training step's passes).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcsf -o run --output-format csv -- python3 tools/sub_pmc.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "asr-transformer_amd"))

import bench  # noqa: E402

r = bench.sub_rooflines(64, 249, 512, 8, 2048, 0.1)
print(json.dumps({k: {f: r[k].get(f) for f in ("us", "frac", "us_warm", "frac_warm")} for k in r}), flush=True)
