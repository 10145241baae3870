"""Band kernel A/B at the representation's Cout 128 shapes (64->128 stem, 128->128) and the Cout 256
shapes, isolated launches timed with HIP events (MZBA_LIB selects the build). usage: python tools/ab_band128.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_conv import run  # noqa: E402

for cin, cout in ((64, 128), (128, 128), (128, 256), (256, 256)):
    print(json.dumps({"lib": os.path.basename(os.environ.get("MZBA_LIB", "libmzba.so")), **run(4096, 16, 20, cin, cout, 3, "band", iters=30)}))
