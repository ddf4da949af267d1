"""GPU train transform microbenchmark (dev tool): the resize/crop/flip/normalise kernel alone and
with a two-op AutoAugment sub-policy, B = 256 CIFAR images into conv1's patch rows. LCCLIP_LIB
selects another build for A/Bs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
for r in range(3):
    print(bench.time_train_transform(256, dev, reps=50), flush=True)
