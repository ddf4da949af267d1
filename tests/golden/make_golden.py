"""Generate tests/golden/tiny_clip.npz from the CPU oracle (oracle/clip_oracle.py).

The reference ships no golden vectors and could not be executed in this environment
(SURVEY.md §8(c)), so these fixtures are produced by the oracle restatement, which is itself pinned
by the reference's known answers in tests/test_oracle.py. They freeze the oracle's behaviour
(so later edits to it are caught) and travel to the GPU box, where the HIP path is compared
against them without recomputing anything on the CPU.

Contents (tiny ViT config: width 128 / 2 heads / 2 layers / 64x64 images, 17 tokens; text width
64 / 1 head / 2 layers / 77 tokens / vocab 512; embed 64):
  sd/<name>                      union state dict (backbone + LoRA + adapter params, nonzero PEFT)
  images, tokens, labels         inputs (B = 2, C = 3)
  <method>/{probs,img_f,txt_f,loss}        fp32 reference outputs, method in vanilla/lora/adapter
  <method>/bf16/{probs,img_f,txt_f}        same with the MI355X path's bf16 rounding points
  <method>/grad/<name>, <method>/new/<name> PEFT gradients and the params after one AdamW step
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import clip_oracle as o  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tiny_clip.npz")


def build():
    torch.manual_seed(0)
    cfg = o.TINY
    sd = {}
    for method in ("vanilla", "lora", "adapter"):
        sd.update(o.synthetic_state_dict(cfg, method, "both", seed=1234))
    images = o.synthetic_images(2, cfg.image_resolution, seed=0)
    tokens = o.synthetic_tokens(3, cfg.context_length, seed=0, vocab=cfg.vocab_size)
    labels = torch.tensor([2, 0])
    out = {"images": images, "tokens": tokens, "labels": labels}
    for k, v in sd.items():
        out["sd/" + k] = v
    for method in ("vanilla", "lora", "adapter"):
        names = o.param_shapes(cfg, method, "both").keys()
        p = {k: sd[k] for k in names}
        loss, probs, fi, ft, grads, new = o.train_step(images, tokens, labels, p, cfg, method, "both")
        out[f"{method}/probs"] = probs
        out[f"{method}/img_f"] = fi
        out[f"{method}/txt_f"] = ft
        out[f"{method}/loss"] = loss.reshape(1)
        for k, g in grads.items():
            out[f"{method}/grad/{k}"] = g
            out[f"{method}/new/{k}"] = new[k]
        with torch.no_grad():
            pb, ib, tb = o.adapter_clip_forward(images, tokens, p, cfg, method, "both", rt=o.round_bf16)
        out[f"{method}/bf16/probs"] = pb
        out[f"{method}/bf16/img_f"] = ib
        out[f"{method}/bf16/txt_f"] = tb
    return {k: v.detach().numpy() for k, v in out.items()}


if __name__ == "__main__":
    arrays = build()
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: {len(arrays)} arrays, {os.path.getsize(OUT) / 1e6:.2f} MB")
