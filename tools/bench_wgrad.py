"""Adapter weight-gradient microbenchmark (dev tool): lc_adapter_wgrad (dWu, dbu, dWd, dbd in one
gemm_tn_wide launch) at the ViT-B/16 step shape M = 50 432, D = 768; HIP-event timing, algorithmic
bytes (gout, z, h, dpre read once) / time. LC_TN_WALKERS overrides the walkers per launch
ONLY in a diagnostic build (make DIAG=1, selected with LCLIB=<that .so>): the production library
ignores schedule environment variables, so the tool refuses them without LCLIB."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

if os.environ.get("LC_TN_WALKERS") and not os.environ.get("LCLIB"):
    raise SystemExit("LC_TN_WALKERS needs a DIAG=1 build selected with LCLIB (the production library "
                     "ignores it, and the result would be mislabelled)")
if os.environ.get("LCLIB"):  # an experimental build of the library
    _lib.load(os.path.join(ROOT, os.environ["LCLIB"]))

dev = torch.device("cuda:0")
M, D = int(os.environ.get("M", 50432)), 768
g = torch.randn(M, D, device=dev).to(torch.bfloat16)
z = torch.randn(M, D, device=dev).to(torch.bfloat16)
h = torch.randn(M, 64, device=dev).to(torch.bfloat16)
dp = torch.randn(M, 64, device=dev).to(torch.bfloat16)
dWu = torch.zeros(D, 64, device=dev)
dWd = torch.zeros(64, D, device=dev)
dbu = torch.zeros(D, device=dev)
dbd = torch.zeros(64, device=dev)
for _ in range(3):
    ops.adapter_wgrad(g, h, z, dp, 0.1, dWu, dbu, dWd, dbd)
reps = 20
from lcclip._lib import call, ptr, stream_of  # noqa: E402


def atomics():
    call("lc_adapter_wgrad", stream_of(g), M, D, ptr(g), g.stride(0), ptr(h), ptr(z), z.stride(0),
         ptr(dp), 0.1, ptr(dWu), ptr(dbu), ptr(dWd), ptr(dbd))


nbytes = (g.numel() + z.numel() + h.numel() + dp.numel()) * 2
for name, fn in (("two-stage", lambda: ops.adapter_wgrad(g, h, z, dp, 0.1, dWu, dbu, dWd, dbd)),
                 ("atomics", atomics)):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    print(f"{name:9s} walkers={os.environ.get('LC_TN_WALKERS', 'cu')} M={M}: {us:.1f} us  "
          f"{nbytes / us / 1e3:.0f} GB/s", flush=True)
