"""AutoAugment kernel debug (dev tool): a failing op chain, op by op, GPU vs oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from oracle import clip_oracle as o  # noqa: E402
from lcclip.transforms import autoaugment  # noqa: E402
from tests.test_autoaug_gpu import images  # noqa: E402

dev = torch.device("cuda:0")
x = images(8, 32, 32, seed=3)
chain = [("Solarize", 113.33333587646484), ("AutoContrast", 0.0)]
for k in range(1, len(chain) + 1):
    got = autoaugment(x.to(dev), chain[:k]).cpu()
    ref = o.autoaugment(x, chain[:k])
    bad = (got != ref).nonzero()
    print(chain[:k], "mismatches", len(bad))
    for idx in bad[:8].tolist():
        n, c, i, j = idx
        print("  at", idx, "got", round(float(got[n, c, i, j]) * 255), "ref", round(float(ref[n, c, i, j]) * 255))
    if len(bad):
        n, c = bad[0][0].item(), bad[0][1].item()
        s = (o.autoaugment(x, chain[:1]) * 255).round()[n, c]
        print("  solarized chan min/max", s.min().item(), s.max().item())
        g1 = (autoaugment(x.to(dev), chain[:1]).cpu() * 255).round()[n, c]
        print("  gpu solarized chan min/max", g1.min().item(), g1.max().item())
