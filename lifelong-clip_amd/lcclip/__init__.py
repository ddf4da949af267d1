"""lcclip — MI355X-native (gfx950) CLIP dual-encoder PEFT training path, a drop-in for the
model surface of qcNPU/LifeLong-CLIP (models/adapter_clip.py, models/clip/). All arithmetic on
the path runs in liblcclip.so (HIP kernels, C ABI in include/lc_clip.h); there is no CPU or ATen
fallback."""
import os as _os

# HIP hardware queues per process (HIP's default is 4). The training step keeps the main stream,
# the text-tower stream and the PEFT weight-gradient stream busy at once, and with a process
# group up RCCL adds its own: at 4 queues two of them share one and stop overlapping (one-rank
# RCCL step 8164-8249 img/s vs 9284 at 8 queues, plain step 9373; profiles/r05/b/). So a value
# below 8 (HIP's 4, which some environments export) is raised to 8; a higher one is kept. Read
# when the HIP runtime initialises, so this only takes effect if lcclip is imported first.
try:
    if int(_os.environ.get("GPU_MAX_HW_QUEUES", "0")) < 8:
        _os.environ["GPU_MAX_HW_QUEUES"] = "8"
except ValueError:
    _os.environ["GPU_MAX_HW_QUEUES"] = "8"
from ._lib import LcError, load as load_library
from .adapter_clip import AdapterCLIP, freeze_backbone
from .clip_loader import available_models, load
from .model import CLIP, build_model
from .trainer import OnlineTrainer, remap_labels

__all__ = ["AdapterCLIP", "CLIP", "OnlineTrainer", "LcError", "available_models", "build_model",
           "freeze_backbone", "load", "load_library", "remap_labels"]
