"""ctypes binding of liblcclip.so (the C ABI declared in include/lc_clip.h).

The product path has no fallback: if the library is missing or a GPU is not present, every
op raises. Tensors cross the boundary as raw device pointers + sizes; the stream is torch's
current HIP stream on the tensor's device.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_long, c_ulonglong, c_void_p

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblcclip.so")

P = c_void_p
# name -> argtypes (restype is always c_int); mirrors include/lc_clip.h
SIGNATURES = {
    "lc_gemm_nt": [P, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_float, P, c_long, P,
                   c_long, P, c_long],
    "lc_gemm_nt_ws": [P, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_float, P, c_long,
                      P, c_long, P, c_long, P, c_long],
    "lc_gemm_nt_fp8": [P, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_long, P, c_long,
                       P, c_float, P, c_long, P, c_long, P, c_long, P, c_long, P, c_long],
    "lc_quant_fp8": [P, c_long, c_int, P, c_int, c_long, c_long, P, c_long, P, c_long],
    "lc_gemm_set_tile": [c_int],
    "lc_gemm_set_streamk": [c_int],
    "lc_gemm_set_debug": [P],
    "lc_adapter_bwd_set_form": [c_int],
    "lc_attn_bwd_set_form": [c_int],
    "lc_gemm_tn": [P, c_int, c_int, c_int, P, c_long, P, c_long, c_float, P, c_long, P, c_float],
    "lc_gemm_tn_ws": [P, c_int, c_int, c_int, P, c_long, P, c_long, c_float, P, c_long, P, c_float,
                      P, c_long],
    "lc_layernorm_fwd": [P, c_int, c_int, P, c_long, P, P, P, P, c_int, c_long, P, P],
    "lc_layernorm_fwd_fp8": [P, c_int, c_int, P, c_long, P, P, P, P, c_long, P, P, P, c_long, P,
                             c_long],
    "lc_layernorm_bwd": [P, c_int, c_int, P, c_int, c_long, P, c_long, P, P, P, P, P, P, c_long, P],
    "lc_layernorm_bwd_fp8": [P, c_int, c_int, P, c_int, c_long, P, c_long, P, P, P, P, P, P, c_long,
                             P, P, c_long, P, c_long],
    "lc_patchify": [P, c_int, c_int, c_int, P, P],
    "lc_vit_assemble": [P, c_int, c_int, c_int, P, P, P, P],
    "lc_vit_embed_ln": [P, c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P],
    "lc_text_embed": [P, c_int, c_int, c_int, P, P, P, P],
    "lc_eot_rows": [P, c_int, c_int, P, P],
    "lc_attn_fwd": [P, c_int, c_int, c_int, P, c_long, P, c_long, P, c_int],
    "lc_attn_bwd": [P, c_int, c_int, c_int, P, c_long, P, P, c_long, P, P, c_long, c_int],
    "lc_attn_bwd_fp8": [P, c_int, c_int, c_int, P, c_long, P, P, c_long, P, P, c_long, P, c_long,
                        c_int],
    "lc_train_transform": [P, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, c_int, P,
                           P, c_int, c_int, c_int, P],
    "lc_autoaugment": [P, c_int, c_int, c_int, c_int, P, P, c_int, P, P],
    "lc_autoaugment_ws": [P, c_int, c_int, c_int, c_int, P, P, c_int, P, P, P, c_long],
    "lc_cast_bf16": [P, c_long, P, P],
    "lc_merge_weight": [P, c_int, c_int, c_int, P, P, P, c_float, P, P],
    "lc_cast_weights_bf16": [P, c_int, P, P, P, P, P],
    "lc_merge_weights_bf16": [P, c_int, P, P, P, P, P, P, P, P, P],
    "lc_lora_grad": [P, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, P, c_float, P, P],
    "lc_lora_grad_ws": [P, c_int, c_int, c_int, c_int, P, c_long, P, c_long, P, c_long, P, c_long,
                        c_float, P, P, P, c_long],
    "lc_adapter_fwd": [P, c_int, c_int, P, c_long, P, P, P, P, c_float, c_float, c_ulonglong, P, P,
                       P, c_long, P],
    "lc_adapter_ln_fwd": [P, c_int, c_int, P, c_long, P, P, P, P, c_float, c_float, c_ulonglong,
                          P, P, P, c_long, P, P, P, P, c_long, P, P],
    "lc_adapter_bwd": [P, c_int, c_int, P, c_long, P, P, P, c_float, c_float, P, P, c_long],
    "lc_adapter_wgrad": [P, c_int, c_int, P, c_long, P, P, c_long, P, c_float, P, P, P, P],
    "lc_adapter_wgrad_ws": [P, c_int, c_int, P, c_long, P, P, c_long, P, c_float, P, P, P, P, P,
                            c_long],
    "lc_check_finite": [P, c_long, P, P],
    "lc_adamw": [P, c_long, P, P, P, P, c_float, c_float, c_float, c_float, c_float, c_int, P, P],
    "lc_counter_add": [P, c_int, P, c_long],
    "lc_adam_step_advance": [P, P, P],
    "lc_l2norm_rows": [P, c_int, c_int, P, c_long, P, P],
    "lc_clip_head": [P, c_int, c_int, c_int, P, P, P, P, P, P, P],
    "lc_head_logits": [P, c_int, c_int, c_int, P, P, P, P, P],
    "lc_softmax_bwd_rows": [P, c_int, c_int, P, P, P],
    "lc_head_feat_grad": [P, c_int, c_int, c_int, P, c_long, c_long, P, P, P, P, P, P],
    "lc_grad_pow2_normalize": [P, c_long, P, P, c_int],
    "lc_add_unscaled": [P, c_long, P, P, P],
    "lc_device_cu_count": [c_int, P],
    "lc_stream_create_cumask": [c_int, c_int, c_int, c_int, P],
    "lc_stream_destroy": [P],
}

# the IEEE-half (text tower) forms: same arguments (include/lc_clip.h, "IEEE-half storage")
F16_ENTRY_POINTS = ("lc_gemm_nt", "lc_gemm_nt_ws", "lc_gemm_tn", "lc_gemm_tn_ws",
                    "lc_layernorm_fwd", "lc_layernorm_bwd", "lc_attn_fwd", "lc_attn_bwd",
                    "lc_attn_bwd_set_form",
                    "lc_cast_bf16", "lc_merge_weight", "lc_cast_weights_bf16",
                    "lc_merge_weights_bf16", "lc_lora_grad", "lc_lora_grad_ws", "lc_adapter_fwd",
                    "lc_adapter_ln_fwd", "lc_adapter_bwd", "lc_adapter_wgrad",
                    "lc_adapter_wgrad_ws", "lc_patchify", "lc_vit_embed_ln")
SIGNATURES.update({n + "_f16": SIGNATURES[n] for n in F16_ENTRY_POINTS})
# the image tower's half residual stream (include/lc_clip.h "x16"): the f32 forms' arguments
SIGNATURES.update({n + "_x16": SIGNATURES[n] for n in (
    "lc_layernorm_fwd", "lc_layernorm_bwd", "lc_vit_embed_ln", "lc_adapter_ln_fwd",
    "lc_layernorm_fwd_fp8", "lc_layernorm_bwd_fp8")})
SIGNATURES["lc_layernorm_bwd_g16"] = SIGNATURES["lc_layernorm_bwd"]
SIGNATURES["lc_adapter_wgrad_ws_unscaled"] = SIGNATURES["lc_adapter_wgrad_ws"] + [P]
SIGNATURES["lc_adapter_wgrad_ws_unscaled_g16"] = SIGNATURES["lc_adapter_wgrad_ws_unscaled"]
SIGNATURES["lc_adapter_bwd_g16"] = SIGNATURES["lc_adapter_bwd"]
SIGNATURES["lc_lora_grad_ws_unscaled"] = SIGNATURES["lc_lora_grad_ws"] + [P]

_lib = None


class LcError(RuntimeError):
    pass


def load(path: str = None):
    """Load liblcclip.so and declare every entry point. Raises if anything is missing.
    LCCLIP_LIB=<path> selects another build of the same library (A/B experiments)."""
    global _lib
    if _lib is not None:
        return _lib
    if path is None:
        path = os.environ.get("LCCLIP_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise LcError(f"liblcclip.so not built at {path}; run `python __graft_entry__.py build` "
                      "(there is no CPU fallback)")
    lib = ctypes.CDLL(path)
    ab = path != LIB_PATH  # an older A/B build may lack newer entry points: those stay unbound
    for name, argtypes in SIGNATURES.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)  # AttributeError if the symbol is missing
        fn.argtypes = argtypes
        fn.restype = c_int
    _lib = lib
    return lib


def exported_symbols(path: str = LIB_PATH):
    lib = ctypes.CDLL(path)
    return {n for n in SIGNATURES if hasattr(lib, n)}


def ptr(t):
    if t is None:
        return None
    return c_void_p(t.data_ptr())


def stream_of(t: torch.Tensor):
    if not t.is_cuda:
        raise LcError("lcclip ops require tensors on a HIP device (no CPU fallback)")
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        kind = {-1: "invalid argument / shape", -2: "kernel launch failed"}.get(rc, "error")
        raise LcError(f"{name} returned {rc} ({kind})")
