"""models/clip/clip_loader.py:83-139 restated for an offline MI355X box.

load(name_or_path): a local checkpoint is read with torch.load(weights_only=True) (state dict, or
{'state_dict': ...} with a 'module.' prefix, clip_loader.py:130-135) and built by
model.build_model. A known architecture name builds that architecture with the reference's
random initialisation instead of downloading (there is no network; clip_loader.py:108-109 would
fetch from openaipublic). TorchScript archives are not accepted (loading one executes code).
"""
from __future__ import annotations

import os

import torch

from .model import CLIP, build_model

# CLIP architectures the reference's _MODELS table names (clip_loader.py:17-32), ViT only.
ARCHITECTURES = {
    "ViT-B/16": dict(embed_dim=512, image_resolution=224, vision_layers=12, vision_width=768,
                     vision_patch_size=16, context_length=77, vocab_size=49408,
                     transformer_width=512, transformer_heads=8, transformer_layers=12),
    "ViT-B/32": dict(embed_dim=512, image_resolution=224, vision_layers=12, vision_width=768,
                     vision_patch_size=32, context_length=77, vocab_size=49408,
                     transformer_width=512, transformer_heads=8, transformer_layers=12),
}


def available_models():
    return list(ARCHITECTURES)


def load(name: str, device=None, jit: bool = False, design_details=None, arch_overrides=None):
    design_details = dict(design_details or {})
    if jit:
        raise ValueError("TorchScript CLIP archives are not supported; pass jit=False")
    if os.path.isfile(name):
        sd = torch.load(name, map_location="cpu", weights_only=True)
        if "state_dict" in sd:
            sd = {k[7:] if k.startswith("module.") else k: v for k, v in sd["state_dict"].items()}
        model = build_model(sd, design_details)
    elif name in ARCHITECTURES or arch_overrides is not None:
        cfg = dict(ARCHITECTURES.get(name, {}))
        cfg.update(arch_overrides or {})
        model = CLIP(design_details=design_details, **cfg)
        for p in model.parameters():
            p.data = p.data.float()
        model = model.eval()
    else:
        raise RuntimeError(f"Model {name} not found; available models = {available_models()}")
    if device is not None:
        model = model.to(device)
    return model
