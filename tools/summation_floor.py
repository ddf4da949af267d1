"""How far apart two evaluations of the SAME rounded algorithm land when only their summation
order / accumulator precision differs (dev tool, CPU only: the oracle). The backward-faithful
rounding oracle (round_bf16_fwd_bwd image tower, round_f16_fwd_bwd text tower) is evaluated with
fp32 accumulation and with fp64 accumulation — the same rounding points, the same rounded
values wherever no rounding boundary is crossed. Their gradient distance is the floor any
implementation of that arithmetic (the HIP path's MFMA accumulation order included) can be
held to on this step; the ill-conditioned adapter down-projection gradients amplify it
(DESIGN.md §2).

    python tools/summation_floor.py METHOD B C SEED      # e.g. adapter 32 10 81
"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import clip_oracle as o  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def cos(a, b):
    return F.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()


def main():
    method = sys.argv[1]
    B, C, seed = (int(a) for a in sys.argv[2:5])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfg = o.VIT_B16
    sd = o.synthetic_state_dict(cfg, method, "both", seed=seed)
    img = o.synthetic_images(B, 224, seed=seed + 1)
    tok = o.synthetic_tokens(C, 77, seed=seed + 2)
    y = torch.arange(B) % C
    kw = dict(rt=o.round_bf16_fwd_bwd, rt_text=o.round_f16_fwd_bwd)
    g32 = o.train_step(img, tok, y, sd, cfg, method, "both")[4]
    ga = o.train_step(img, tok, y, sd, cfg, method, "both", **kw)[4]
    ln = o.layer_norm
    o.layer_norm = lambda x, w, b, eps=1e-5: F.layer_norm(x, (x.shape[-1],), w, b, eps)
    try:
        sd64 = {k: v.double() for k, v in sd.items()}
        gb = o.train_step(img.double(), tok, y, sd64, cfg, method, "both", **kw)[4]
    finally:
        o.layer_norm = ln
    cat = lambda d: torch.cat([d[n].flatten().double() for n in g32])  # noqa: E731
    worst = min(g32, key=lambda n: cos(ga[n].double(), gb[n]))
    print(f"{method} B={B} C={C}: rounding oracle fp32-accumulated vs fp64-accumulated: "
          f"flat {rel(cat(ga), cat(gb)):.3e}, min cos {cos(ga[worst].double(), gb[worst]):.5f} "
          f"({worst}); each vs the fp32 algorithm: {rel(cat(ga), cat(g32)):.3e} / "
          f"{rel(cat(gb), cat(g32)):.3e}", flush=True)


if __name__ == "__main__":
    main()
