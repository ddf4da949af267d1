"""Per-tensor PEFT gradient error vs the fp32 oracle as a function of the class count C
(adapter, ViT-B/16, B = 4) — localises a class-count-dependent gradient error (dev tool)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from oracle import clip_oracle as o  # noqa: E402
from lcclip import OnlineTrainer  # noqa: E402
from lcclip.adapter_clip import AdapterCLIP, set_adapter_dropout  # noqa: E402

dev = torch.device("cuda:0")
torch.set_num_threads(16)
method = os.environ.get("METHOD", "adapter")
cfg = o.TINY if os.environ.get("TINY") else o.VIT_B16
res = cfg.image_resolution
for C in [int(c) for c in os.environ.get("CS", "16,64,65,100").split(",")]:
    B = int(os.environ.get("B", 4))
    sd = o.synthetic_state_dict(cfg, method, "both", seed=71)
    img = o.synthetic_images(B, res, seed=72)
    tok = o.synthetic_tokens(C, 77, seed=73, vocab=cfg.vocab_size)
    y = torch.arange(B) % C
    loss32, p32, i32, t32, g32, _ = o.train_step(img, tok, y, sd, cfg, method, "both")
    w = set_adapter_dropout(AdapterCLIP.from_state_dict(sd, method, "both", device=dev), 0.0)
    tr = OnlineTrainer(w)
    loss, probs = tr.forward_backward(img.to(dev), y.to(dev), tok.to(dev))
    named = dict(w.model.named_parameters())
    rows = []
    for n, g in g32.items():
        gg = tr.grads[named[n]].float().cpu()
        rows.append((((gg - g).norm() / g.norm()).item(), g.norm().item(), gg.norm().item(), n))
    rows.sort(reverse=True)
    img_r = max(r[0] for r in rows if r[3].startswith("visual"))
    txt_r = max(r[0] for r in rows if not r[3].startswith("visual"))
    print(f"C={C}: loss {loss.item():.6f} vs {loss32.item():.6f}  img max rel {img_r:.4f}  txt max rel {txt_r:.4f}")
    for r in rows[:6]:
        print(f"   {r[0]:.4f}  |g32| {r[1]:.3e}  |gpu| {r[2]:.3e}  {r[3]}")
