"""lcclip — MI355X-native (gfx950) CLIP dual-encoder PEFT training path, a drop-in for the
model surface of qcNPU/LifeLong-CLIP (models/adapter_clip.py, models/clip/). All arithmetic on
the path runs in liblcclip.so (HIP kernels, C ABI in include/lc_clip.h); there is no CPU or ATen
fallback."""
from ._lib import LcError, load as load_library
from .adapter_clip import AdapterCLIP, freeze_backbone
from .clip_loader import available_models, load
from .model import CLIP, build_model
from .trainer import OnlineTrainer, remap_labels

__all__ = ["AdapterCLIP", "CLIP", "OnlineTrainer", "LcError", "available_models", "build_model",
           "freeze_backbone", "load", "load_library", "remap_labels"]
