"""Attention fwd/bwd microbenchmark at the ViT-B/16 B=256 image shape and the text shape (dev tool).

Prints one line per kernel: average ms over REPS launches, achieved TFLOP/s (algorithmic, unpadded
L: fwd 2 matmuls, bwd 5 matmuls of L x L x 64 per (sequence, head)). FORMS=1,2,3 times each
lc_attn_bwd_set_form form of the backward in turn (default: the automatic one)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

REPS = int(os.environ.get("REPS", 20))
dev = torch.device("cuda:0")


def run(name, n, L, H, causal):
    D = H * 64
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(n * L, 3 * D, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    O = torch.empty(n * L, D, device=dev, dtype=torch.bfloat16)
    dO = (torch.randn(n * L, D, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    lse = torch.empty(n * H, L, device=dev)
    dqkv = torch.empty_like(qkv)
    for f, fl, tag in ((lambda: ops.attn_fwd(qkv, O, lse, n, L, H, causal), 2, "fwd"),
                       (lambda: ops.attn_bwd(qkv, O, dO, lse, dqkv, n, L, H, causal), 5, "bwd")):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / REPS
        flops = fl * 2.0 * n * H * L * L * 64 * (0.5 if causal else 1.0)
        print(f"{name:6s} {tag} n={n} L={L} H={H}: {ms * 1e3:8.1f} us  {flops / ms / 1e9:7.1f} TFLOP/s",
              flush=True)


for form in [int(f) for f in os.environ.get("FORMS", "0").split(",")]:
    if _lib.load().lc_attn_bwd_set_form(form) != 0:
        raise SystemExit(f"lc_attn_bwd_set_form({form}) rejected")
    print(f"-- backward form {form}", flush=True)
    run("image", int(os.environ.get("B", 256)), 197, 12, False)
    run("text", int(os.environ.get("C", 100)), 77, 8, True)
