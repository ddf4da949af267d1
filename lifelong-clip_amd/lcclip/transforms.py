"""GPU train transform of the online step.

Reference: methods/_trainer.py:212-242 builds

    Compose([(x*255).type(uint8), AutoAugment(policy), x.float()/255,           # 'autoaug'
             Resize((224, 224)), RandomCrop(224, padding=4), RandomHorizontalFlip(),
             Normalize(mean, std)])

(policy: CIFAR10 for 'cifar*' datasets, IMAGENET for '*imagenet*', SVHN for 'svhn',
_trainer.py:217-228) and methods/adapter_clip.py:81 applies it to the whole batch tensor on the
GPU. On a batched tensor torchvision draws ONE set of random parameters per call, so the whole
batch shares the sub-policy, the crop offset and the flip; they are drawn here in torchvision's
order (AutoAugment.get_params: torch.randint(len(policies)), torch.rand(2), torch.randint(2, (2,));
RandomCrop.get_params: i then j by torch.randint over [0, 2*padding]; RandomHorizontalFlip:
torch.rand(1) < 0.5).

Two kernels (transform.hip): lc_autoaugment applies the drawn sub-policy's active ops to the
uint8-quantised batch (one workgroup per image, the image in LDS), and lc_train_transform does
the bilinear resize, the padded crop, the flip and the normalisation in a single pass over the
output (or, with no augmentation op active, the uint8 round trip itself). layout="patches" writes
conv1's bf16 im2col rows directly ([n*196, 768] for ViT-B/16), which ImageTower.forward accepts in
place of an image batch, so the f32 224x224 batch never touches HBM.

The AutoAugment policy tables, magnitude bins and op semantics restate torchvision 0.16.2
(requirements.yaml:269; transforms/autoaugment.py, transforms/_functional_tensor.py), which is not
installed here: parity is pinned against the oracle's independent restatement
(oracle/clip_oracle.py autoaugment), not against torchvision itself ("parity unpinned").
"""
from __future__ import annotations

import ctypes
import math

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


# torchvision.transforms.AutoAugmentPolicy tables: (op, probability, magnitude bin or None)
AUTOAUG_POLICIES = {
    "cifar10": [
        (("Invert", 0.1, None), ("Contrast", 0.2, 6)),
        (("Rotate", 0.7, 2), ("TranslateX", 0.3, 9)),
        (("Sharpness", 0.8, 1), ("Sharpness", 0.9, 3)),
        (("ShearY", 0.5, 8), ("TranslateY", 0.7, 9)),
        (("AutoContrast", 0.5, None), ("Equalize", 0.9, None)),
        (("ShearY", 0.2, 7), ("Posterize", 0.3, 7)),
        (("Color", 0.4, 3), ("Brightness", 0.6, 7)),
        (("Sharpness", 0.3, 9), ("Brightness", 0.7, 9)),
        (("Equalize", 0.6, None), ("Equalize", 0.5, None)),
        (("Contrast", 0.6, 7), ("Sharpness", 0.6, 5)),
        (("Color", 0.7, 7), ("TranslateX", 0.5, 8)),
        (("Equalize", 0.3, None), ("AutoContrast", 0.4, None)),
        (("TranslateY", 0.4, 3), ("Sharpness", 0.2, 6)),
        (("Brightness", 0.9, 6), ("Color", 0.2, 8)),
        (("Solarize", 0.5, 2), ("Invert", 0.0, None)),
        (("Equalize", 0.2, None), ("AutoContrast", 0.6, None)),
        (("Equalize", 0.2, None), ("Equalize", 0.6, None)),
        (("Color", 0.9, 9), ("Equalize", 0.6, None)),
        (("AutoContrast", 0.8, None), ("Solarize", 0.2, 8)),
        (("Brightness", 0.1, 3), ("Color", 0.7, 0)),
        (("Solarize", 0.4, 5), ("AutoContrast", 0.9, None)),
        (("TranslateY", 0.9, 9), ("TranslateY", 0.7, 9)),
        (("AutoContrast", 0.9, None), ("Solarize", 0.8, 3)),
        (("Equalize", 0.8, None), ("Invert", 0.1, None)),
        (("TranslateY", 0.7, 9), ("AutoContrast", 0.9, None)),
    ],
    "imagenet": [
        (("Posterize", 0.4, 8), ("Rotate", 0.6, 9)),
        (("Solarize", 0.6, 5), ("AutoContrast", 0.6, None)),
        (("Equalize", 0.8, None), ("Equalize", 0.6, None)),
        (("Posterize", 0.6, 7), ("Posterize", 0.6, 6)),
        (("Equalize", 0.4, None), ("Solarize", 0.2, 4)),
        (("Equalize", 0.4, None), ("Rotate", 0.8, 8)),
        (("Solarize", 0.6, 3), ("Equalize", 0.6, None)),
        (("Posterize", 0.8, 5), ("Equalize", 1.0, None)),
        (("Rotate", 0.2, 3), ("Solarize", 0.6, 8)),
        (("Equalize", 0.6, None), ("Posterize", 0.4, 6)),
        (("Rotate", 0.8, 8), ("Color", 0.4, 0)),
        (("Rotate", 0.4, 9), ("Equalize", 0.6, None)),
        (("Equalize", 0.0, None), ("Equalize", 0.8, None)),
        (("Invert", 0.6, None), ("Equalize", 1.0, None)),
        (("Color", 0.6, 4), ("Contrast", 1.0, 8)),
        (("Rotate", 0.8, 8), ("Color", 1.0, 2)),
        (("Color", 0.8, 8), ("Solarize", 0.8, 7)),
        (("Sharpness", 0.4, 7), ("Invert", 0.6, None)),
        (("ShearX", 0.6, 5), ("Equalize", 1.0, None)),
        (("Color", 0.4, 0), ("Equalize", 0.6, None)),
        (("Equalize", 0.4, None), ("Solarize", 0.2, 4)),
        (("Solarize", 0.6, 5), ("AutoContrast", 0.6, None)),
        (("Invert", 0.6, None), ("Equalize", 1.0, None)),
        (("Color", 0.6, 4), ("Contrast", 1.0, 8)),
        (("Equalize", 0.8, None), ("Equalize", 0.6, None)),
    ],
    "svhn": [
        (("ShearX", 0.9, 4), ("Invert", 0.2, None)),
        (("ShearY", 0.9, 8), ("Invert", 0.7, None)),
        (("Equalize", 0.6, None), ("Solarize", 0.6, 6)),
        (("Invert", 0.9, None), ("Equalize", 0.6, None)),
        (("Equalize", 0.6, None), ("Rotate", 0.9, 3)),
        (("ShearX", 0.9, 4), ("AutoContrast", 0.8, None)),
        (("ShearY", 0.9, 8), ("Invert", 0.4, None)),
        (("ShearY", 0.9, 5), ("Solarize", 0.2, 6)),
        (("Invert", 0.9, None), ("AutoContrast", 0.8, None)),
        (("Equalize", 0.6, None), ("Rotate", 0.9, 3)),
        (("ShearX", 0.9, 4), ("Solarize", 0.3, 3)),
        (("ShearY", 0.8, 8), ("Invert", 0.7, None)),
        (("Equalize", 0.9, None), ("TranslateY", 0.6, 6)),
        (("Invert", 0.9, None), ("Equalize", 0.6, None)),
        (("Contrast", 0.3, 3), ("Rotate", 0.8, 4)),
        (("Invert", 0.8, None), ("TranslateY", 0.0, 2)),
        (("ShearY", 0.7, 6), ("Solarize", 0.4, 8)),
        (("Invert", 0.6, None), ("Rotate", 0.8, 4)),
        (("ShearY", 0.3, 7), ("TranslateX", 0.9, 3)),
        (("ShearX", 0.1, 6), ("Invert", 0.6, None)),
        (("Solarize", 0.7, 2), ("TranslateY", 0.6, 7)),
        (("ShearY", 0.8, 4), ("Invert", 0.8, None)),
        (("ShearX", 0.7, 9), ("TranslateY", 0.8, 3)),
        (("ShearY", 0.8, 5), ("AutoContrast", 0.7, None)),
        (("ShearX", 0.7, 2), ("Invert", 0.1, None)),
    ],
}


def policy_for_dataset(name):
    """methods/_trainer.py:217-228."""
    if "cifar" in name:
        return "cifar10"
    if "imagenet" in name:
        return "imagenet"
    if "svhn" in name:
        return "svhn"
    return None


def augmentation_space(num_bins, height, width):
    """AutoAugment._augmentation_space: op -> (magnitude bins (f32, as torch computes them),
    signed)."""
    return {
        "ShearX": (torch.linspace(0.0, 0.3, num_bins), True),
        "ShearY": (torch.linspace(0.0, 0.3, num_bins), True),
        "TranslateX": (torch.linspace(0.0, 150.0 / 331.0 * width, num_bins), True),
        "TranslateY": (torch.linspace(0.0, 150.0 / 331.0 * height, num_bins), True),
        "Rotate": (torch.linspace(0.0, 30.0, num_bins), True),
        "Brightness": (torch.linspace(0.0, 0.9, num_bins), True),
        "Color": (torch.linspace(0.0, 0.9, num_bins), True),
        "Contrast": (torch.linspace(0.0, 0.9, num_bins), True),
        "Sharpness": (torch.linspace(0.0, 0.9, num_bins), True),
        "Posterize": (8 - (torch.arange(num_bins) / ((num_bins - 1) / 4)).round().int(), False),
        "Solarize": (torch.linspace(255.0, 0.0, num_bins), False),
        "AutoContrast": (torch.tensor(0.0), False),
        "Equalize": (torch.tensor(0.0), False),
        "Invert": (torch.tensor(0.0), False),
    }


def draw_autoaugment(policy, height, width, generator=None):
    """AutoAugment.forward's draws (one per call, shared by the batch) -> the active ops as
    [(op_name, magnitude)] in application order."""
    pol = AUTOAUG_POLICIES[policy]
    tid = int(torch.randint(len(pol), (1,), generator=generator).item())
    probs = torch.rand((2,), generator=generator)
    signs = torch.randint(2, (2,), generator=generator)
    space = augmentation_space(10, height, width)
    out = []
    for i, (op, p, mid) in enumerate(pol[tid]):
        if probs[i] <= p:
            mags, signed = space[op]
            mag = float(mags[mid].item()) if mid is not None else 0.0
            if signed and signs[i] == 0:
                mag *= -1.0
            out.append((op, mag))
    return out


def _inverse_affine(center, angle, translate, scale, shear):
    """torchvision.transforms.functional._get_inverse_affine_matrix (doubles)."""
    rot = math.radians(angle)
    sx, sy = math.radians(shear[0]), math.radians(shear[1])
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    m = [v / scale for v in m]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty)
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty)
    m[2] += cx
    m[5] += cy
    return m


def _affine_grid_theta(m, width, height):
    """_gen_affine_grid's rescaled theta: f32(m) / f32(0.5 * size), column x then y."""
    t = torch.tensor(m, dtype=torch.float32)
    sx, sy = torch.tensor(0.5 * width, dtype=torch.float32), torch.tensor(0.5 * height,
                                                                        dtype=torch.float32)
    return [float(t[0] / sx), float(t[1] / sx), float(t[2] / sx),
            float(t[3] / sy), float(t[4] / sy), float(t[5] / sy)]


# largest C*H*W whose two working images fit the LDS form of lc_autoaugment (transform.hip)
AUTOAUG_LDS_ELEMS = 12288

# lc_autoaugment op codes (transform.hip AA_*)
_AA = {"Invert": 0, "Brightness": 1, "Color": 2, "Contrast": 3, "Sharpness": 4, "Posterize": 5,
       "Solarize": 6, "AutoContrast": 7, "Equalize": 8}
_AA_AFFINE = 9


def autoaug_kernel_ops(ops, height, width):
    """[(op, magnitude)] -> (codes, params[6 per op]) for lc_autoaugment (_apply_op restated)."""
    codes, params = [], []
    for op, mag in ops:
        p = [0.0] * 6
        if op in ("Brightness", "Color", "Contrast", "Sharpness"):
            ratio = 1.0 + mag
            p[0] = float(torch.tensor(ratio, dtype=torch.float32))
            p[1] = float(torch.tensor(1.0 - ratio, dtype=torch.float32))
            if op == "Sharpness":
                k = torch.ones(3, 3)
                k[1, 1] = 5.0
                k /= k.sum()
                p[2], p[3] = float(k[0, 0]), float(k[1, 1])
            codes.append(_AA[op])
        elif op == "Posterize":
            codes.append(_AA[op])
            p[0] = float((-int(2 ** (8 - int(mag)))) & 0xFF)
        elif op == "Solarize":
            codes.append(_AA[op])
            p[0] = float(torch.tensor(mag, dtype=torch.float32))
        elif op in ("AutoContrast", "Equalize", "Invert"):
            codes.append(_AA[op])
        else:  # affine ops, nearest, zero fill
            if op == "ShearX":
                m = _inverse_affine([-0.5 * width, -0.5 * height], 0.0, [0.0, 0.0], 1.0,
                                    [math.degrees(math.atan(mag)), 0.0])
            elif op == "ShearY":
                m = _inverse_affine([-0.5 * width, -0.5 * height], 0.0, [0.0, 0.0], 1.0,
                                    [0.0, math.degrees(math.atan(mag))])
            elif op == "TranslateX":
                m = _inverse_affine([0.0, 0.0], 0.0, [float(int(mag)), 0.0], 1.0, [0.0, 0.0])
            elif op == "TranslateY":
                m = _inverse_affine([0.0, 0.0], 0.0, [0.0, float(int(mag))], 1.0, [0.0, 0.0])
            elif op == "Rotate":  # F.rotate passes -angle (functional.py rotate)
                m = _inverse_affine([0.0, 0.0], -mag, [0.0, 0.0], 1.0, [0.0, 0.0])
            else:
                raise ValueError(f"unknown AutoAugment op {op}")
            codes.append(_AA_AFFINE)
            p = _affine_grid_theta(m, width, height)
        params.extend(p)
    return codes, params


def autoaugment(x, ops):
    """The active AutoAugment ops on the GPU: x f32 [n, C, H, W] in [0, 1] -> f32
    (uint8-quantised, augmented) / 255 (lc_autoaugment)."""
    if x.dim() != 4 or x.dtype != torch.float32:
        raise ValueError("autoaugment expects an f32 [n, C, H, W] batch")
    x = x.contiguous()
    n, C, H, W = x.shape
    codes, params = autoaug_kernel_ops(ops, H, W)
    out = torch.empty_like(x)
    cb = (ctypes.c_int * max(len(codes), 1))(*codes)
    pb = (ctypes.c_float * max(len(params), 1))(*params)
    if C * H * W <= AUTOAUG_LDS_ELEMS:  # the image fits the kernel's LDS form
        call("lc_autoaugment", stream_of(x), n, C, H, W, ptr(x), ptr(out), len(codes),
             ctypes.cast(cb, ctypes.c_void_p), ctypes.cast(pb, ctypes.c_void_p))
    else:  # ImageNet-sized: working images in HBM (out + a scratch image per input)
        ws = torch.empty(n * C * H * W, dtype=torch.int32, device=x.device)
        call("lc_autoaugment_ws", stream_of(x), n, C, H, W, ptr(x), ptr(out), len(codes),
             ctypes.cast(cb, ctypes.c_void_p), ctypes.cast(pb, ctypes.c_void_p), ptr(ws),
             ws.numel() * 4)
    return out


class TrainTransform:
    """`self.train_transform` of methods/_trainer.py:236-242 on the GPU.

    x: f32 [n, C, H, W] on the GPU with ToTensor values in [0, 1] (the dataset's transform,
    _trainer.py:197). Returns the normalised [n, C, S, S] f32 batch, or with
    layout="patches" the bf16 patch rows of conv1 (see module docstring)."""

    def __init__(self, mean, std, inp_size=224, padding=4, autoaug=True, patch=16,
                 generator=None, policy=None):
        if len(mean) != len(std) or not 1 <= len(mean) <= 4:
            raise ValueError("mean/std must have one entry per channel (1..4)")
        self.mean = [float(m) for m in mean]
        self.std = [float(s) for s in std]
        self.inp_size = int(inp_size)
        self.padding = int(padding)
        self.autoaug = bool(autoaug)
        self.patch = int(patch)
        self.generator = generator
        # the AutoAugment policy of the 'autoaug' branch (None: the uint8 round trip only)
        self.policy = policy if autoaug else None

    @classmethod
    def for_dataset(cls, name, **kw):
        mean, std = DATASET_STATS[name]
        kw.setdefault("policy", policy_for_dataset(name))
        return cls(mean, std, **kw)

    def draw(self, height=32, width=32):
        """One call's random parameters in torchvision's order: the AutoAugment sub-policy's
        active ops (when a policy is set), then RandomCrop.get_params, then
        RandomHorizontalFlip -> (ops, crop_i, crop_j, flip)."""
        ops = (draw_autoaugment(self.policy, height, width, self.generator)
               if self.policy is not None else [])
        span = 2 * self.padding + 1
        i = int(torch.randint(0, span, (1,), generator=self.generator))
        j = int(torch.randint(0, span, (1,), generator=self.generator))
        flip = bool(torch.rand(1, generator=self.generator) < 0.5)
        return ops, i, j, flip

    def __call__(self, x, params=None, layout="nchw"):
        if params is None:
            params = self.draw(x.shape[-2], x.shape[-1])
        if len(params) == 3:  # (crop_i, crop_j, flip): no augmentation op
            params = ([],) + tuple(params)
        ops, i, j, flip = params
        if x.dim() != 4 or x.dtype != torch.float32:
            raise ValueError("TrainTransform expects an f32 [n, C, H, W] batch")
        n, C, H, W = x.shape
        if C != len(self.mean):
            raise ValueError(f"batch has {C} channels, mean/std have {len(self.mean)}")
        x = x.contiguous()
        quantize = int(self.autoaug)
        if ops:
            if not self.autoaug:
                raise ValueError("AutoAugment ops need the autoaug branch")
            x = autoaugment(x, ops)  # uint8 round trip + ops, written back as k / 255
            quantize = 0
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
             ctypes.cast(std, ctypes.c_void_p), quantize, lay, P, ptr(out))
        return out
