"""Yardstick (dev tool): torch.mm (hipBLASLt on ROCm) on the step's plain GEMM shapes, bf16,
random data, HIP-event timing; prints TF/s next to the lc_gemm_nt ping-pong kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import ops  # noqa: E402

dev = torch.device("cuda:0")
M = 50432
for name, N, K in (("qkv_fwd", 2304, 768), ("fc1_fwd", 3072, 768), ("fc2_fwd", 768, 3072),
                   ("qkv_dx", 768, 2304), ("out_fwd", 768, 768)):
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    res = {}
    for tag, fn in (("torch.mm", lambda: torch.mm(A, B.t(), out=o)),
                    ("lc_gemm_nt", lambda: ops.gemm_nt(A, B, ops.EPI_BF16, o))):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        res[tag] = (us, 2 * M * N * K / us / 1e6)
    print(f"{name:8s} N={N:5d} K={K:5d} | " + " | ".join(f"{k}: {v[0]:7.1f} us {v[1]:6.0f} TF"
                                                        for k, v in res.items()), flush=True)
