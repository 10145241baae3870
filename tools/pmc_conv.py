"""Single-shape driver for PMC passes on the dominant kernel at the bench's B: run under
`rocprofv3 --pmc FETCH_SIZE --kernel-trace` (and WRITE_SIZE in a separate pass).
  pmc_conv.py B            conv_lat 3x3 256->256 (one latent residual conv)
  pmc_conv.py B tower N    tower_kernel, N residual blocks (the bench's dyn/pred tower)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import torch  # noqa: E402
from mzba import _lib as L  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
H, W, C = 4, 5, 256
if len(sys.argv) > 2 and sys.argv[2] == "tower":
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 14
    x = torch.randn(B * H * W * C, device="cuda").to(torch.bfloat16)
    out = torch.empty_like(x)
    wf = (torch.randn(2 * nb * C * 9 * C + 8 * 64 * 8, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(2 * nb * C, device="cuda")
    nws = L.lib().mzba_tower_ws_bytes(B)
    ws = torch.zeros(max(nws, 16), dtype=torch.uint8, device="cuda")
    for _ in range(20):
        L.call("mzba_tower", L.ptr(x), H * W * C, None, 0, L.ptr(out), L.ptr(wf), L.ptr(b), nb, B, L.ptr(ws), nws,
               L.stream())
    torch.cuda.synchronize()
    print("done tower", B, nb)
    sys.exit(0)
x = torch.randn(B * H * W * C, device="cuda").to(torch.bfloat16)
res = torch.randn(B * H * W * C, device="cuda").to(torch.bfloat16)
out = torch.empty(B * H * W * C, device="cuda", dtype=torch.bfloat16)
w = (torch.randn(C * 9 * C + 8 * 64 * 8, device="cuda") * 0.02).to(torch.bfloat16)
b = torch.zeros(C, device="cuda")
for _ in range(20):
    L.call("mzba_conv_lat", L.ptr(x), H * W * C, None, 0, L.ptr(w), L.ptr(b), None, None, 0, L.ptr(res), L.ptr(out),
           B, H, W, C, C, 3, 1, L.stream())
torch.cuda.synchronize()
print("done", B)
