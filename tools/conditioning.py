"""Where the PEFT-gradient distance from fp32 comes from, per tower (dev tool, CPU only: the
oracle). The oracle's rounding hooks are straight-through (the forward is rounded, the backward
runs in fp32), so each line is the gradient distance that the named FORWARD precision alone
causes, for the adapter step of tests/test_model_gpu.py::_step_vs_oracle.

    python tools/conditioning.py B C SEED          # e.g. 32 10 81 (config 2's C), 4 100 71

Lines: bf16 everywhere (the pre-r4 GPU path), fp16 everywhere (the reference's autocast,
methods/adapter_clip.py:87), and one tower in bf16 with the other in fp16 or fp32.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import clip_oracle as o  # noqa: E402


def round_fp16(x):
    r = x.detach().to(torch.float16).to(x.dtype)
    return x + (r - x).detach()


HOOK = {"fp32": o.identity, "bf16": o.round_bf16, "fp16": round_fp16}


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def cos(a, b):
    return torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()


def main():
    B, C, seed = (int(a) for a in sys.argv[1:4])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfg, method = o.VIT_B16, "adapter"
    sd = o.synthetic_state_dict(cfg, method, "both", seed=seed)
    img = o.synthetic_images(B, 224, seed=seed + 1)
    tok = o.synthetic_tokens(C, 77, seed=seed + 2)
    y = torch.arange(B) % C
    g32 = o.train_step(img, tok, y, sd, cfg, method, "both")[4]
    cat = lambda d: torch.cat([d[n].flatten() for n in g32])  # noqa: E731
    orig_ei, orig_et = o.encode_image, o.encode_text

    def run(img_p, txt_p):
        def ei(img_, p, cfg_, m, pe, rt, masks=None):
            return orig_ei(img_, p, cfg_, m, pe, HOOK[img_p], masks)

        def et(tok_, p, cfg_, m, pe, rt, masks=None):
            return orig_et(tok_, p, cfg_, m, pe, HOOK[txt_p], masks)
        o.encode_image, o.encode_text = ei, et
        try:
            g = o.train_step(img, tok, y, sd, cfg, method, "both")[4]
        finally:
            o.encode_image, o.encode_text = orig_ei, orig_et
        w = min((cos(g[n], g32[n]), rel(g[n], g32[n]), n) for n in g32)
        print(f"image {img_p}, text {txt_p}:  flat rel {rel(cat(g), cat(g32)):.4f}   worst tensor "
              f"cosine {w[0]:.4f} (rel {w[1]:.3f}, {w[2]})", flush=True)

    print(f"ViT-B/16 adapter both towers, B = {B}, C = {C}, seed {seed}: PEFT-gradient distance "
          "from the fp32 oracle with the forward rounded as named (straight-through)")
    for ip, tp in (("bf16", "bf16"), ("fp16", "fp16"), ("bf16", "fp16"), ("fp16", "bf16"),
                   ("bf16", "fp32"), ("fp32", "bf16")):
        run(ip, tp)


if __name__ == "__main__":
    main()
