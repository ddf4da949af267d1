import os, sys
sys.path[:0] = ["/root/repo", "/root/repo/lifelong-clip_amd"]
import torch
from lcclip import _lib, ops
dev = torch.device("cuda:0")
lib = _lib.load()
for form in (1, 3):
    lib.lc_attn_bwd_set_form(form)
    for n in (128, 256, 384, 512, 1024):
        H, L = 2, 197
        D = H * 64
        qkv = (torch.randn(n * L, 3 * D, device=dev) * 0.5).to(torch.bfloat16)
        O = torch.empty(n * L, D, device=dev, dtype=torch.bfloat16)
        dO = (torch.randn(n * L, D, device=dev) * 0.1).to(torch.bfloat16)
        lse = torch.empty(n * H, L, device=dev)
        dqkv = torch.empty_like(qkv)
        ops.attn_fwd(qkv, O, lse, n, L, H, False)
        f = lambda: ops.attn_bwd(qkv, O, dO, lse, dqkv, n, L, H, False)
        f(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): f()
        e1.record(); torch.cuda.synchronize()
        print(f"form {form} items {n*H:5d}: {e0.elapsed_time(e1)/20*1e3:8.1f} us", flush=True)
