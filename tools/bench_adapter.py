"""Adapter / LayerNorm streaming-kernel microbenchmark at the ViT-B/16 B=256 shape (dev tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import ops  # noqa: E402

M, D = int(os.environ.get("M", 50432)), int(os.environ.get("D", 768))
dev = torch.device("cuda:0")
bf = torch.bfloat16
z = torch.randn(M, D, device=dev).to(bf)
Wd = (torch.randn(64, D, device=dev) * 0.03).to(bf)
Wu = (torch.randn(D, 64, device=dev) * 0.1).to(bf)
bd = torch.randn(64, device=dev) * 0.1
bu = torch.randn(D, device=dev) * 0.1
resid = torch.randn(M, D, device=dev)
x = torch.empty(M, D, device=dev)
h = torch.empty(M, 64, device=dev, dtype=bf)
dpre = torch.empty(M, 64, device=dev, dtype=bf)
dz = torch.empty(M, D, device=dev, dtype=bf)
WuT, WdT = Wu.t().contiguous(), Wd.t().contiguous()
w = torch.randn(D, device=dev)
dWu, dbu = torch.zeros(D, 64, device=dev), torch.zeros(D, device=dev)
dWd, dbd = torch.zeros(64, D, device=dev), torch.zeros(64, device=dev)
y = torch.empty(M, D, device=dev, dtype=bf)
mean = torch.empty(M, device=dev)
rstd = torch.empty(M, device=dev)


def t(fn, reps=20):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


cases = {
    "adapter_fwd keep=1": (lambda: ops.adapter_fwd(z, Wd, bd, Wu, bu, 0.1, 1.0, 7, resid, x, h),
                           M * D * (2 + 4 + 4) + M * 128),
    "adapter_fwd keep=.9": (lambda: ops.adapter_fwd(z, Wd, bd, Wu, bu, 0.1, 0.9, 7, resid, x, h),
                            M * D * (2 + 4 + 4) + M * 128),
    "adapter_bwd": (lambda: ops.adapter_bwd(z, h, WuT, WdT, 0.1, 1.0, dpre, dz), M * D * 4 + M * 256),
    "adapter_wgrad": (lambda: ops.adapter_wgrad(z, h, z, dpre, 0.1, dWu, dbu, dWd, dbd),
                      M * D * 4 + M * 256),
    "gemm_tn x2 (old)": (lambda: (ops.gemm_tn(z, h, dWu, alpha=0.1, colsum=dbu, colsum_scale=0.1),
                                  ops.gemm_tn(dpre, z, dWd, colsum=dbd)), M * D * 4 + M * 256),
    "ln_fwd bf16": (lambda: ops.layernorm_fwd(resid, w, w, y, mean, rstd), M * D * 6),
}
for name, (fn, nbytes) in cases.items():
    us = t(fn)
    print(f"{name:22s} {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
