"""lc_adapter_ln_fwd_x16 (the half residual stream's fused adapter + LayerNorm) at the ViT-B/16
B = 256 step shape, standalone (dev tool): HIP-event time per launch and algorithmic bytes / time.
LCCLIP_LIB=<.so> times another build (e.g. an ADLN_KO store-knockout diagnostic build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import ops  # noqa: E402

M, D = int(os.environ.get("M", 50432)), 768
dev = torch.device("cuda:0")
BF, H16 = torch.bfloat16, torch.float16
torch.manual_seed(0)
z = torch.randn(M, D, device=dev).to(BF)
Wd = (torch.randn(64, D, device=dev) * D ** -0.5).to(BF)
Wu = (torch.randn(D, 64, device=dev) * 0.125).to(BF)
bd, bu = torch.randn(64, device=dev) * 0.1, torch.randn(D, device=dev) * 0.1
x = torch.randn(M, D, device=dev).to(H16)
xo = torch.empty(M, D, device=dev, dtype=H16)
h = torch.empty(M, 64, device=dev, dtype=BF)
gam, bet = torch.randn(D, device=dev), torch.randn(D, device=dev)
y = torch.empty(M, D, device=dev, dtype=BF)
m, r = torch.empty(M, device=dev), torch.empty(M, device=dev)


def launch():
    ops.adapter_ln_fwd(z, Wd, bd, Wu, bu, 0.1, 0.9, 7, x, xo, h, gam, bet, y, m, r)


for _ in range(5):
    launch()
reps = int(os.environ.get("REPS", 50))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = None
for _ in range(3):
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    best = us if best is None else min(best, us)
nbytes = M * (D * 2 * 4 + 64 * 2 + 8)  # z, resid in; x_out, y out (2 B each); h; mean / rstd
print(f"adapter_ln_fwd_x16 M={M} D={D}: {best:.1f} us  {nbytes / best / 1e6:.2f} TB/s", flush=True)
