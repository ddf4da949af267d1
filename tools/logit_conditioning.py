"""Which bf16 rounding drives the logits' max |d|/s from fp32 (dev tool, CPU only: the oracle,
forward). d = logits - logits_fp32, s = exp(logit_scale) (tests/parity.py). Lines: the
bf16-rounding oracle as the GPU path rounds, the same with the towers' tails (ln_post /
ln_final output and the projection GEMM) in f32, and with one tower entirely in f32.

    python tools/logit_conditioning.py METHOD B C SEED    # e.g. adapter 32 10 81, lora 16 16 61
"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import clip_oracle as o  # noqa: E402
from parity import logit_errors  # noqa: E402


def hook(tail32=False):
    def rt(x):
        return o.round_bf16(x)
    if tail32:
        rt.tail = o.identity
    return rt


def main():
    method = sys.argv[1]
    B, C, seed = (int(a) for a in sys.argv[2:5])
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfg = o.VIT_B16
    sd = o.synthetic_state_dict(cfg, method, "both", seed=seed)
    img = o.synthetic_images(B, 224, seed=seed + 1)
    tok = o.synthetic_tokens(C, 77, seed=seed + 2)
    ls = math.exp(sd["logit_scale"].item())
    with torch.no_grad():
        fi = {}
        ft = {}
        for name, rt in (("fp32", o.identity), ("bf16", hook()), ("bf16_tail32", hook(True))):
            fi[name] = o.encode_image(img, sd, cfg, method, "both", rt)
            ft[name] = o.encode_text(tok, sd, cfg, method, "both", rt)

    def lg(i, t):
        i = i / i.norm(dim=-1, keepdim=True)
        t = t / t.norm(dim=-1, keepdim=True)
        return ls * i @ t.t()
    ref = lg(fi["fp32"], ft["fp32"])
    for a, b in (("bf16", "bf16"), ("bf16_tail32", "bf16_tail32"), ("fp32", "bf16"),
                 ("bf16", "fp32"), ("fp32", "bf16_tail32"), ("bf16_tail32", "fp32")):
        mx, rms = logit_errors(lg(fi[a], ft[b]), ref, ls)
        print(f"{method} B={B} C={C}  image {a:12s} text {b:12s}  max {mx:.3e}  rms {rms:.3e}",
              flush=True)


if __name__ == "__main__":
    main()
