"""MaPLe (models/maple.py, BASELINE config 5) on the MI355X vs the CPU oracle
(oracle.clip_oracle.maple_forward): learned text context in the text tower's input rows, the
shared visual context appended before ln_pre (L = 197 + 3 at ViT-B/16), deep compound prompts
replacing rows at layers 1..2 of both towers; logits and the gradients of every prompt-learner
parameter through CE.

Parity unpinned against the reference itself. Tolerances as
tests/test_model_gpu.py: logits in cosine units < 2e-3 vs fp32 (< 1e-3 vs the bf16-rounding
oracle); gradients rel-norm < 6e-2 vs fp32 (bf16 activations through two frozen towers)."""
import math
import os

import pytest
import torch
import torch.nn.functional as F

from oracle import clip_oracle as o

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def record(**kw):
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
    with open(os.path.join(root, "gpurun_out", "parity_metrics.jsonl"), "a") as f:
        f.write(json.dumps(kw) + "\n")


def run_case(cfg, sd, mp, img, tok, y, dev, tag):
    from lcclip.maple import MaPLe
    with torch.no_grad():
        l32 = o.maple_forward(img, tok, sd, cfg, mp)
        l16 = o.maple_forward(img, tok, sd, cfg, mp, rt=o.round_bf16)
    mpg = {k: v.clone().requires_grad_(True) for k, v in mp.items()}
    F.cross_entropy(o.maple_forward(img, tok, sd, cfg, mpg), y).backward()

    m = MaPLe.from_state_dict(sd, device=dev)
    params = dict(m.named_parameters())
    with torch.no_grad():
        for k, name in o.MAPLE_TO_MODULE.items():
            params[name].copy_(mp[k])
    m.set_tokenized_prompts(tok.to(dev))
    logits = m(img.to(dev))
    F.cross_entropy(logits, y.to(dev)).backward()
    torch.cuda.synchronize()
    ls = math.exp(sd["logit_scale"].item())
    met = dict(cos_err_vs_fp32=((logits.detach().cpu() - l32).abs().max() / ls).item(),
               cos_err_vs_bf16=((logits.detach().cpu() - l16).abs().max() / ls).item())
    for k, name in o.MAPLE_TO_MODULE.items():
        met[f"grad_{k}_rel"] = rel(params[name].grad, mpg[k].grad)
    record(test=tag, **met)
    assert met["cos_err_vs_fp32"] < 2e-3 and met["cos_err_vs_bf16"] < 1e-3, met
    for k in o.MAPLE_TO_MODULE:
        assert met[f"grad_{k}_rel"] < 6e-2, (k, met)
    # only the prompt learner trains
    assert {n for n, p in m.named_parameters() if p.requires_grad} == set(
        o.MAPLE_TO_MODULE.values())


def test_maple_tiny(dev):
    cfg = o.TINY_MAPLE
    run_case(cfg, o.synthetic_state_dict(cfg, seed=41), o.maple_params(cfg, seed=2),
             o.synthetic_images(3, cfg.image_resolution, seed=6),
             o.synthetic_tokens(4, 77, seed=6, vocab=cfg.vocab_size), torch.tensor([0, 2, 3]),
             dev, "maple_tiny")


def test_maple_vit_b16_shapes(dev):
    """ViT-B/16 + 12-layer text tower: image L = 200, B = 2, C = 4."""
    cfg = o.VIT_B16
    run_case(cfg, o.synthetic_state_dict(cfg, seed=43), o.maple_params(cfg, seed=3),
             o.synthetic_images(2, 224, seed=7), o.synthetic_tokens(4, 77, seed=7),
             torch.tensor([1, 3]), dev, "maple_vit_b16")
