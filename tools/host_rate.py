"""Host-side launch rate of the bench step (dev tool): wall time of trainer.step() calls as they
return (no sync: the host enqueue cost per step) vs the synchronised step time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from lcclip import AdapterCLIP, OnlineTrainer  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(1234)
model = AdapterCLIP("ViT-B/16", peft_method="adapter", peft_encoder="both", device=dev)
tr = OnlineTrainer(model)
x, tok, y = bench.synthetic_batch(256, 10, dev, seed=100)
for _ in range(5):
    tr.step(x, y, tok)
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    tr.step(x, y, tok)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue {1e3 * (t1 - t0) / n:.2f} ms/step, GPU-complete {1e3 * (t2 - t0) / n:.2f} ms/step",
      flush=True)
