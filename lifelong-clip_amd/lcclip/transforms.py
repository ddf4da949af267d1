"""GPU train transform of the online step.

Reference: methods/_trainer.py:212-242 builds

    Compose([(x*255).type(uint8), AutoAugment(cifar10 policy), x.float()/255,   # 'autoaug'
             Resize((224, 224)), RandomCrop(224, padding=4), RandomHorizontalFlip(),
             Normalize(mean, std)])

and methods/adapter_clip.py:81 applies it to the whole batch tensor on the GPU. On a batched
tensor torchvision draws ONE set of random parameters per call, so the whole batch shares the
crop offset and the flip; they are drawn here in torchvision's order (RandomCrop.get_params: i
then j by torch.randint over [0, 2*padding]; RandomHorizontalFlip: torch.rand(1) < 0.5).

One kernel (lc_train_transform, transform.hip) does the uint8 round trip, the bilinear resize,
the padded crop, the flip and the normalisation in a single pass over the output.
layout="patches" writes conv1's bf16 im2col rows directly ([n*196, 768] for ViT-B/16), which
ImageTower.forward accepts in place of an image batch, so the f32 224x224 batch never touches HBM.
Not applied: the AutoAugment op itself (the quantise/dequantise around it is). It is the
optional part of SURVEY.md §8(f) f2 and is listed as open in DESIGN.md §9.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import call, ptr, stream_of

# datasets/__init__.py:35-58: (mean, std) per dataset
DATASET_STATS = {
    "cifar10": ((0.4914, 0.4822, 0.4465), (0.2470, 0.2435, 0.2616)),
    "cifar100": ((0.5071, 0.4867, 0.4408), (0.2675, 0.2565, 0.2761)),
    "svhn": ((0.4377, 0.4438, 0.4728), (0.1980, 0.2010, 0.1970)),
    "tinyimagenet": ((0.4802, 0.4481, 0.3975), (0.2302, 0.2265, 0.2262)),
    "imagenet": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
    "imagenet-r": ((0.485, 0.456, 0.406), (0.229, 0.224, 0.225)),
}


class TrainTransform:
    """`self.train_transform` of methods/_trainer.py:236-242 on the GPU.

    x: f32 [n, C, H, W] on the GPU with ToTensor values in [0, 1] (the dataset's transform,
    _trainer.py:197). Returns the normalised [n, C, S, S] f32 batch, or with
    layout="patches" the bf16 patch rows of conv1 (see module docstring)."""

    def __init__(self, mean, std, inp_size=224, padding=4, autoaug=True, patch=16,
                 generator=None):
        if len(mean) != len(std) or not 1 <= len(mean) <= 4:
            raise ValueError("mean/std must have one entry per channel (1..4)")
        self.mean = [float(m) for m in mean]
        self.std = [float(s) for s in std]
        self.inp_size = int(inp_size)
        self.padding = int(padding)
        self.autoaug = bool(autoaug)
        self.patch = int(patch)
        self.generator = generator

    @classmethod
    def for_dataset(cls, name, **kw):
        mean, std = DATASET_STATS[name]
        return cls(mean, std, **kw)

    def draw(self):
        """(crop_i, crop_j, flip): RandomCrop.get_params then RandomHorizontalFlip."""
        span = 2 * self.padding + 1
        i = int(torch.randint(0, span, (1,), generator=self.generator))
        j = int(torch.randint(0, span, (1,), generator=self.generator))
        flip = bool(torch.rand(1, generator=self.generator) < 0.5)
        return i, j, flip

    def __call__(self, x, params=None, layout="nchw"):
        if params is None:
            params = self.draw()
        i, j, flip = params
        if x.dim() != 4 or x.dtype != torch.float32:
            raise ValueError("TrainTransform expects an f32 [n, C, H, W] batch")
        n, C, H, W = x.shape
        if C != len(self.mean):
            raise ValueError(f"batch has {C} channels, mean/std have {len(self.mean)}")
        x = x.contiguous()
        R, P = self.inp_size, self.patch
        if layout == "nchw":
            out = torch.empty(n, C, R, R, dtype=torch.float32, device=x.device)
            lay = 0
        elif layout == "patches":
            if R % P:
                raise ValueError("inp_size must be a multiple of the patch size")
            g = R // P
            out = torch.empty(n * g * g, C * P * P, dtype=torch.bfloat16, device=x.device)
            lay = 1
        else:
            raise ValueError("layout must be 'nchw' or 'patches'")
        mean = (ctypes.c_float * C)(*self.mean)
        std = (ctypes.c_float * C)(*self.std)
        call("lc_train_transform", stream_of(x), n, C, H, W, ptr(x), R, self.padding, int(i),
             int(j), int(bool(flip)), ctypes.cast(mean, ctypes.c_void_p),
             ctypes.cast(std, ctypes.c_void_p), int(self.autoaug), lay, P, ptr(out))
        return out
