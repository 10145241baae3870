"""Band kernel width A/B (mzba_conv_band_set_xt 10 vs 5) at the acting loop's representation shapes,
isolated launches timed with HIP events. usage: python tools/bench_band_xt.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_conv import run  # noqa: E402
from mzba import _lib as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for xt in (10, 5):
    L.call("mzba_conv_band_set_xt", xt)
    for cin, cout in ((256, 256), (128, 128), (128, 256)):
        r = run(B, 16, 20, cin, cout, 3, "band", iters=20)
        print(json.dumps({"xt": xt, **r}))
L.call("mzba_conv_band_set_xt", 5)
