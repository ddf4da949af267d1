"""AdapterCLIP — drop-in for models/adapter_clip.py:14-137 of qcNPU/LifeLong-CLIP.

Same constructor arguments, attributes (.model, .dtype, .text_tokens, .current_class_names,
.prompt_template) and forward contract: forward(image, text_tokens=None) ->
(probs [B,C], image_features [B,E], text_features [C,E]) with probs = softmax(logits)
(adapter_clip.py:94-100). `.module` returns self so the reference trainer's
`self.custom_clip.module...` calls work on one GPU (Q4).

Tokenisation (the CLIP BPE, models/clip/tokenizer.py) is a CPU producer of int64 ids and is out
of this build's scope: pass `tokenizer=` (a callable text -> list[int] without
SOT/EOT) to use class names, or hand set_token()/forward() precomputed token ids.
"""
from __future__ import annotations

from typing import List, Union

import torch
import torch.nn as nn

from . import autograd as lc_autograd
from . import clip_loader

SOT_TOKEN = 49406
EOT_TOKEN = 49407


class AdapterCLIP(nn.Module):
    def __init__(self, model_name, peft_method="adapter", peft_encoder="both", device=None,
                 tokenizer=None, arch_overrides=None, text_precision="fp16",
                 image_precision="bf16"):
        super().__init__()
        self.device = device
        design_details = {
            "method": peft_method,
            "peft_encoder": peft_encoder,
            "ffn_num": 64,
            "lora_alpha": 1,
            "lora_r": 4,
        }
        self.model = clip_loader.load(model_name, device=device, jit=False,
                                      design_details=design_details, arch_overrides=arch_overrides)
        self.text_tokens = None
        self.current_class_names = []
        self.dtype = self.model.dtype
        self.prompt_template = "a bad photo of a {}."
        self._tokenizer = tokenizer
        self.set_text_precision(text_precision)
        self.set_image_precision(image_precision)

    def set_image_precision(self, precision):
        """The image tower's 16-bit storage: 'bf16' (default; BASELINE config 2 names bf16 for
        the throughput configuration: half residual stream, bf16 GEMM / attention operands) or
        'fp16' (the reference's own arithmetic, torch.cuda.amp.autocast fp16 at
        methods/adapter_clip.py:87: IEEE-half GEMM / attention operands, an f32 residual stream,
        and the backward on a per-call power-of-two gradient scale, the GradScaler's role at
        :93). Extension of the reference surface, like set_text_precision."""
        dt = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(precision)
        if dt is None:
            raise ValueError("image_precision must be 'fp16' or 'bf16'")
        self.model.visual.tower.stack.set_storage(dt)
        self.image_precision = precision
        return self

    def set_text_precision(self, precision):
        """The text tower's 16-bit storage: 'fp16' (default; IEEE half, the precision the
        reference's towers run at under torch.cuda.amp.autocast, methods/adapter_clip.py:87) or
        'bf16'. The image tower stays bf16 (BASELINE config 2). Extension of the reference
        surface: the reference has one autocast switch for the whole model."""
        dt = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(precision)
        if dt is None:
            raise ValueError("text_precision must be 'fp16' or 'bf16'")
        self.model.transformer.engine.set_storage(dt)
        self.text_precision = precision
        return self

    @classmethod
    def from_state_dict(cls, state_dict, peft_method="adapter", peft_encoder="both", device=None,
                        tokenizer=None, text_precision="fp16", image_precision="bf16"):
        """Build from an in-memory CLIP state dict (the path clip_loader.load takes for a local
        checkpoint file, clip_loader.py:116-135)."""
        from .model import build_model
        self = cls.__new__(cls)
        nn.Module.__init__(self)
        self.device = device
        dd = {"method": peft_method, "peft_encoder": peft_encoder, "ffn_num": 64, "lora_alpha": 1,
              "lora_r": 4}
        self.model = build_model(dict(state_dict), dd)
        if device is not None:
            self.model = self.model.to(device)
        self.text_tokens = None
        self.current_class_names = []
        self.dtype = self.model.dtype
        self.prompt_template = "a bad photo of a {}."
        self._tokenizer = tokenizer
        self.set_image_precision(image_precision)
        return self.set_text_precision(text_precision)

    @property
    def module(self):
        return self

    def tokenize(self, texts: Union[str, List[str]], context_length: int = 77) -> torch.LongTensor:
        """adapter_clip.py:108-137 (requires a tokenizer callable)."""
        if self._tokenizer is None:
            raise RuntimeError("no BPE tokenizer configured; pass tokenizer= or token ids")
        if isinstance(texts, str):
            texts = [texts]
        all_tokens = [[SOT_TOKEN] + list(self._tokenizer(t)) + [EOT_TOKEN] for t in texts]
        result = torch.zeros(len(all_tokens), context_length, dtype=torch.long)
        for i, tokens in enumerate(all_tokens):
            tokens = tokens[:context_length]
            result[i, :len(tokens)] = torch.tensor(tokens)
        return result

    def labels_tokenize(self, labels, context_length: int = 77) -> torch.LongTensor:
        """adapter_clip.py:43-74: prompt template applied to each class name."""
        if isinstance(labels, str):
            labels = [labels]
        return self.tokenize([self.prompt_template.format(c) for c in labels], context_length).to(
            self._param_device())

    def _param_device(self):
        return self.model.logit_scale.device

    def encode_image(self, image):
        """adapter_clip.py:76-79 (L2-normalised image features)."""
        return lc_autograd.l2norm_apply(self.model.encode_image(image))

    def update_class_names(self, new_class_names):
        """adapter_clip.py:81-92 (appends unseen names; returns None as the reference does)."""
        for c in new_class_names:
            if c not in self.current_class_names:
                self.current_class_names.append(c)
        return None

    def forward(self, image, text_tokens=None):
        if text_tokens is None:
            text_tokens = self.text_tokens
        img_f = self.model.encode_image(image)
        txt_f = self.model.encode_text(text_tokens)
        probs, image_features, text_features = lc_autograd.head_apply(
            img_f, txt_f, self.model.logit_scale, probs=True)
        return probs, image_features, text_features

    def set_token(self, classnames_or_tokens):
        """adapter_clip.py:102-104; accepts class names (needs a tokenizer) or token ids."""
        if isinstance(classnames_or_tokens, torch.Tensor):
            tokens = classnames_or_tokens.to(self._param_device(), torch.long)
        else:
            tokens = self.labels_tokenize(classnames_or_tokens)
        if "text_tokens" in self._buffers:
            del self._buffers["text_tokens"]
        elif hasattr(self, "text_tokens"):
            del self.text_tokens
        self.register_buffer("text_tokens", tokens)


def set_adapter_dropout(model: nn.Module, p: float):
    """Set the adapter dropout probability (adapter.py:61; 0.1 in the reference). Parity tests use
    p = 0 because a dropout RNG stream cannot be matched bit-exactly."""
    for m in model.modules():
        if m.__class__.__name__ == "Adapter":
            m.dropout = float(p)
    return model


def freeze_backbone(model: nn.Module):
    """methods/adapter_clip.py:117-119: only '*adaptmlp*' / '*lora*' parameters stay trainable."""
    for k, v in model.named_parameters():
        if "adaptmlp" not in k and "lora" not in k:
            v.requires_grad = False
    return model
