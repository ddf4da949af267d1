"""Conditioning of the C = 100 adapter gradients (tests/test_model_gpu.py::
test_adapter_c100_step_vs_oracle, ViT-B/16 both towers, B = 4, C = 100): how far the PEFT
gradients move from fp32 when the FORWARD alone is rounded (the oracle's round_bf16 /
round_fp16 hooks are straight-through: no backward rounding) — bf16 everywhere, fp16 everywhere
(the reference's own precision: fp16 autocast, methods/adapter_clip.py:87), and bf16 at one
rounding site of the text tower at a time (image tower fp32).

CPU only (the oracle); about 3 minutes on 8 threads:
    python tools/c100_conditioning.py > profiles/r03/c100_conditioning.txt
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import clip_oracle as o  # noqa: E402

I, R = o.identity, o.round_bf16


def round_fp16(x):
    r = x.detach().to(torch.float16).to(x.dtype)
    return x + (r - x).detach()


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def cos(a, b):
    return torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfg, method, B, C, seed = o.VIT_B16, "adapter", 4, 100, 71
    sd = o.synthetic_state_dict(cfg, method, "both", seed=seed)
    img = o.synthetic_images(B, 224, seed=seed + 1)
    tok = o.synthetic_tokens(C, 77, seed=seed + 2)
    y = torch.arange(B) % C
    g32 = o.train_step(img, tok, y, sd, cfg, method, "both")[4]
    cat = lambda d: torch.cat([d[n].flatten() for n in g32])  # noqa: E731

    def report(name, g):
        w = min((cos(g[n], g32[n]), rel(g[n], g32[n]), n) for n in g32)
        print(f"{name:48s} flat rel {rel(cat(g), cat(g32)):.4f}   worst tensor cosine {w[0]:.4f} "
              f"(rel {w[1]:.3f}, {w[2]})")

    print(f"ViT-B/16 adapter both towers, B = {B}, C = {C}, seed {seed}; distance of the PEFT "
          "gradients from the fp32 oracle with the forward rounded as named")
    report("bf16 everywhere (the GPU's storage precision)",
           o.train_step(img, tok, y, sd, cfg, method, "both", rt=R)[4])
    report("fp16 everywhere (the reference's autocast)",
           o.train_step(img, tok, y, sd, cfg, method, "both", rt=round_fp16)[4])
    orig_ei, orig_block = o.encode_image, o.block

    def ei(img, p, cfg, method, pe, rt, masks=None):
        return orig_ei(img, p, cfg, method, pe, I, masks)

    def make_block(sites):
        def blk(x, p, pre, n_head, causal, variant, lora_scaling=0.25, rt=I, masks=None):
            if not pre.startswith("transformer."):
                return orig_block(x, p, pre, n_head, causal, variant, lora_scaling, I, masks)
            r = lambda s: R if s in sites else I  # noqa: E731
            h = r("ln")(o.layer_norm(x, p[pre + "ln_1.weight"], p[pre + "ln_1.bias"]))
            a = o.mha(h, p, pre, n_head, causal, None, r("attention"))
            x = x + o.adapter(r("adapter input")(a), p, pre, rt=r("adapter GEMMs"))
            h2 = r("ln")(o.layer_norm(x, p[pre + "ln_2.weight"], p[pre + "ln_2.bias"]))
            f = r("mlp")(o.quick_gelu(o.linear(h2, p[pre + "mlp.c_fc.weight"],
                                                p[pre + "mlp.c_fc.bias"], r("mlp"))))
            m = o.linear(f, p[pre + "mlp.c_proj.weight"], p[pre + "mlp.c_proj.bias"], r("mlp"))
            return x + o.adapter(r("adapter input")(m), p, pre, rt=r("adapter GEMMs"))
        return blk
    try:
        o.encode_image = ei
        for site in ("ln", "attention", "adapter input", "adapter GEMMs", "mlp"):
            o.block = make_block({site})
            report(f"text tower, bf16 at '{site}' only",
                   o.train_step(img, tok, y, sd, cfg, method, "both", rt=I)[4])
    finally:
        o.encode_image, o.block = orig_ei, orig_block


if __name__ == "__main__":
    main()
