"""LoRA weight-gradient microbenchmark (dev tool): ops.lora_grad_1p (one pass over X and dY:
lora_grad1p_kernel + lora_reduce_kernel) at the LoRA step's sites, rank 4, alone on the GPU.
HIP-event timing over 20 launches; algorithmic bytes = X and dY read once. LCLIB selects another
build of the library."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

if os.environ.get("LCLIB"):
    _lib.load(os.path.join(ROOT, os.environ["LCLIB"]))

dev = torch.device("cuda:0")
r, reps = 4, 20
for M in (25216, 50432):
    for N, K in ((2304, 768), (768, 768)):
        X = torch.randn(M, K, device=dev).to(torch.bfloat16)
        dY = torch.randn(M, N, device=dev).to(torch.bfloat16)
        a_pad = torch.zeros(16, K, device=dev, dtype=torch.bfloat16)
        bt_pad = torch.zeros(16, N, device=dev, dtype=torch.bfloat16)
        a_pad[:r] = (torch.randn(r, K, device=dev) * 0.02).to(torch.bfloat16)
        bt_pad[:r] = (torch.randn(r, N, device=dev) * 0.02).to(torch.bfloat16)
        dA = torch.zeros(r, K, device=dev)
        dB = torch.zeros(N, r, device=dev)
        fn = lambda: ops.lora_grad_1p(dY, X, a_pad, bt_pad, r, 2.0, dA, dB)  # noqa: E731
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        nbytes = (X.numel() + dY.numel()) * 2
        print(f"lora_grad_1p M={M} N={N} K={K}: {us:.1f} us  {nbytes / us / 1e3:.0f} GB/s",
              flush=True)
        del X, dY
