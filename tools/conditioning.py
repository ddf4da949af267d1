"""Where the PEFT-gradient distance from fp32 comes from, per tower (dev tool, CPU only: the
oracle). The oracle's rounding hooks are straight-through (the forward is rounded, the backward
runs in fp32), so each line is the gradient distance that the named FORWARD precision alone
causes, for the adapter step of tests/test_model_gpu.py::_step_vs_oracle.

    python tools/conditioning.py B C SEED          # e.g. 32 10 81 (config 2's C), 4 100 71

Lines: bf16 everywhere (the pre-r4 GPU path), fp16 everywhere (the reference's autocast,
methods/adapter_clip.py:87), and one tower in bf16 with the other in fp16 or fp32.

    python tools/conditioning.py B C SEED attn     # both towers bf16, the text tower's attention
                                                   # (QKV output, P, O) at other precisions
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

    if sys.argv[4:] == ["attn"]:
        return text_attention_sites(run_rounded(img, tok, y, sd, cfg, method, g32, cat), B, C, seed)
    print(f"ViT-B/16 adapter both towers, B = {B}, C = {C}, seed {seed}: PEFT-gradient distance "
          "from the fp32 oracle with the forward rounded as named (straight-through)")
    for ip, tp in (("bf16", "bf16"), ("fp16", "fp16"), ("bf16", "fp16"), ("fp16", "bf16"),
                   ("bf16", "fp32"), ("fp32", "bf16")):
        run(ip, tp)


def run_rounded(img, tok, y, sd, cfg, method, g32, cat):
    """Both towers' forward rounded to bf16, with the text attention replaced by `attn`."""
    def go(label, attn):
        orig_mha, orig_ei, orig_et = o.mha, o.encode_image, o.encode_text

        def mha(x, p, pre, n_head, causal, lora_scaling=None, rt=o.identity):
            if not causal:  # the image tower
                return orig_mha(x, p, pre, n_head, causal, lora_scaling, rt)
            return attn(x, p, pre, n_head, rt)

        def ei(img_, p, cfg_, m, pe, rt, masks=None):
            return orig_ei(img_, p, cfg_, m, pe, o.round_bf16, masks)

        def et(tok_, p, cfg_, m, pe, rt, masks=None):
            return orig_et(tok_, p, cfg_, m, pe, o.round_bf16, masks)
        o.mha, o.encode_image, o.encode_text = mha, ei, et
        try:
            g = o.train_step(img, tok, y, sd, cfg, method, "both")[4]
        finally:
            o.mha, o.encode_image, o.encode_text = orig_mha, orig_ei, orig_et
        w = min((cos(g[n], g32[n]), rel(g[n], g32[n]), n) for n in g32)
        print(f"{label:34s} flat rel {rel(cat(g), cat(g32)):.4f}   worst tensor cosine {w[0]:.4f} "
              f"(rel {w[1]:.3f}, {w[2]})", flush=True)
    return go


def text_attention_sites(go, B, C, seed):
    """mha (oracle/clip_oracle.py:284-307) for the text tower with the QKV GEMM output, the
    probabilities P and the attention output O rounded by the named hooks."""
    def attn_with(hq, hp, ho):
        def attn(x, p, pre, n_head, rt):
            N, L, D = x.shape
            qkv = HOOK[hq](o.linear(x, p[pre + "attn.in_proj_weight"], p[pre + "attn.in_proj_bias"], rt))
            q, k, v = (t.reshape(N, L, n_head, D // n_head).permute(0, 2, 1, 3) for t in qkv.chunk(3, dim=-1))
            s = (q @ k.transpose(-1, -2)) * (D // n_head) ** -0.5
            s = s + torch.full((L, L), float("-inf")).triu_(1)
            e = torch.exp(s - s.amax(dim=-1, keepdim=True))
            out = HOOK[ho]((HOOK[hp](e) @ v) / e.sum(dim=-1, keepdim=True))
            out = out.permute(0, 2, 1, 3).reshape(N, L, D)
            return o.linear(out, p[pre + "attn.out_proj.weight"], p[pre + "attn.out_proj.bias"], rt)
        return attn
    print(f"ViT-B/16 adapter both towers, B = {B}, C = {C}, seed {seed}: both towers' forward bf16 "
          "except the text attention's roundings as named (straight-through)")
    for hq, hp, ho in (("bf16", "bf16", "bf16"), ("bf16", "fp16", "bf16"), ("bf16", "fp32", "bf16"),
                       ("bf16", "bf16", "fp16"), ("fp16", "bf16", "bf16"), ("fp16", "fp16", "fp16"),
                       ("fp32", "fp32", "fp32")):
        go(f"text qkv {hq}, P {hp}, O {ho}:", attn_with(hq, hp, ho))


if __name__ == "__main__":
    main()
