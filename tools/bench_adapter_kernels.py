"""Adapter forward / backward kernels at the ViT-B/16 step shape (dev tool): lc_adapter_fwd
(EPI_AD_DOWN + EPI_AD_UP), lc_adapter_bwd (EPI_AD_MASK + EPI_AD_ADD) and the fused adapter +
LayerNorm forward (lc_adapter_ln_fwd), HIP-event timing and algorithmic bytes / time. LC_GEMM_TILE forces a tile family
for the experiment ONLY in a diagnostic build (make DIAG=1, selected with LCLIB=<that .so>): the
production library ignores schedule environment variables, so the tool refuses them without LCLIB."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

if os.environ.get("LC_GEMM_TILE") and not os.environ.get("LCLIB"):
    raise SystemExit("LC_GEMM_TILE needs a DIAG=1 build selected with LCLIB (the production library "
                     "ignores it, and the result would be mislabelled)")
if os.environ.get("LCLIB"):
    _lib.load(os.path.join(ROOT, os.environ["LCLIB"]))
dev = torch.device("cuda:0")
M, D, H = 50432, 768, 64
BF = torch.bfloat16
z = torch.randn(M, D, device=dev).to(BF)
Wd = (torch.randn(H, D, device=dev) * 0.03).to(BF)
Wu = (torch.randn(D, H, device=dev) * 0.03).to(BF)
WuT, WdT = Wu.t().contiguous(), Wd.t().contiguous()
bd, bu = torch.randn(H, device=dev), torch.randn(D, device=dev)
resid = torch.randn(M, D, device=dev)
xout = torch.empty(M, D, device=dev)
h = torch.empty(M, H, device=dev, dtype=BF)
g = torch.randn(M, D, device=dev).to(BF)
dpre = torch.empty(M, H, device=dev, dtype=BF)
dz = torch.empty(M, D, device=dev, dtype=BF)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


fwd = timeit(lambda: ops.adapter_fwd(z, Wd, bd, Wu, bu, 0.1, 0.9, 1234, resid, xout, h))
down = timeit(lambda: ops.adapter_bwd(g, h, WuT, WdT, 0.1, 0.9, dpre, None))
bwd = timeit(lambda: ops.adapter_bwd(g, h, WuT, WdT, 0.1, 0.9, dpre, dz))
up_bytes = (M * D * 4 * 2 + M * D * 2 + M * H * 2)
add_bytes = (M * D * 2 * 2 + M * H * 2)
gamma, beta = torch.randn(D, device=dev), torch.randn(D, device=dev)
y = torch.empty(M, D, device=dev, dtype=BF)
mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
adln = timeit(lambda: ops.adapter_ln_fwd(z, Wd, bd, Wu, bu, 0.1, 0.9, 1234, resid, xout, h, gamma,
                                         beta, y, mean, rstd))
adln_bytes = M * (D * 2 + D * 4 + D * 4 + D * 2 + H * 2 + 8)
print(f"adapter_ln_fwd {adln:.1f} us ({adln_bytes / adln / 1e6:.2f} TB/s)", flush=True)
print(f"tile={os.environ.get('LC_GEMM_TILE', 'auto')} adapter_fwd {fwd:.1f} us | bwd mask {down:.1f} us, "
      f"mask+add {bwd:.1f} us -> add {bwd - down:.1f} us ({add_bytes / (bwd - down) / 1e6:.2f} TB/s); "
      f"up-proj side bytes {up_bytes / 1e6:.0f} MB", flush=True)
