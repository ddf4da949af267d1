"""lcclip — MI355X-native (gfx950) CLIP dual-encoder PEFT training path, a drop-in for the
model surface of qcNPU/LifeLong-CLIP (models/adapter_clip.py, models/clip/). All arithmetic on
the path runs in liblcclip.so (HIP kernels, C ABI in include/lc_clip.h); there is no CPU or ATen
fallback."""
import os as _os

# HIP hardware queues per process (GPU_MAX_HW_QUEUES, read once when the HIP runtime
# initialises; HIP's default is 4). lcclip never changes it: a launcher that wants more queues
# (bench.py raises it to 8 before importing torch) sets it before HIP starts. The value seen at
# import is what OnlineTrainer._merge_side_streams decides from.
HW_QUEUES_AT_IMPORT = _os.environ.get("GPU_MAX_HW_QUEUES")
from ._lib import LcError, load as load_library
from .adapter_clip import AdapterCLIP, freeze_backbone
from .clip_loader import available_models, load
from .model import CLIP, build_model
from .trainer import OnlineTrainer, remap_labels

__all__ = ["AdapterCLIP", "CLIP", "OnlineTrainer", "LcError", "available_models", "build_model",
           "freeze_backbone", "load", "load_library", "remap_labels"]
