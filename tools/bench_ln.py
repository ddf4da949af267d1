"""LayerNorm forward / backward at the ViT-B/16 step shape (dev tool): HIP-event timing and
algorithmic bytes / time. LCCLIP_LIB selects another build for A/Bs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import ops  # noqa: E402

dev = torch.device("cuda:0")
M, D = 50432, 768
x = torch.randn(M, D, device=dev)
w, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
dres = torch.randn(M, D, device=dev)
dx = torch.empty(M, D, device=dev)
dxb = torch.empty(M, D, device=dev, dtype=torch.bfloat16)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


f = timeit(lambda: ops.layernorm_fwd(x, w, b, y, mean, rstd))
bw = timeit(lambda: ops.layernorm_bwd(dy, x, mean, rstd, w, dx, dxb, dres=dres))
fb, bb = M * D * (4 + 2), M * D * (2 + 4 + 4 + 4 + 2)
print(f"lib={os.environ.get('LCCLIP_LIB', 'product')} ln_fwd {f:.1f} us ({fb / f / 1e6:.2f} TB/s) | "
      f"ln_bwd {bw:.1f} us ({bb / bw / 1e6:.2f} TB/s)", flush=True)
