"""MaPLe — drop-in for models/maple.py:17-253 of qcNPU/LifeLong-CLIP (BASELINE config 5:
multi-modal prompt learning, n_ctx = 3, compound prompt depth 3).

Same module tree and parameter names (prompt_learner.{ctx, proj, compound_prompts_text.*,
compound_prompt_projections.*}), buffers (token_prefix, token_suffix), attributes
(image_encoder, text_encoder, logit_scale, dtype, n_ctx, base_clip_model, tokenized_prompts,
current_class_names, prompt_prefix) and forward(image, tokenized_prompts=None, prefix=None,
suffix=None) -> logits. Both towers run on the liblcclip engine with the reference's prompt
semantics (models/maple_clip/model.py:316-401, 522-590): the text input embeddings carry the
learned context at rows 1..n_ctx, the image sequence gets proj(ctx) appended before ln_pre
(L = 197 + n_ctx), and at layers 1..depth-1 the deep prompts overwrite those rows; backward
returns the gradients of every prompt row through the frozen blocks.

Deviations: the image tower computes with bf16 MFMA operands and fp32 accumulation on the half
residual stream (the reference casts the visual prompts to fp16, model.py:374 and :569); the
text tower stores IEEE half (text_precision='fp16', the reference's dtype; 'bf16' optional).
precision='fp8' (BASELINE config 5) runs the image tower's frozen QKV / c_fc / c_proj GEMMs,
forward and input-gradient, as block-scaled e4m3 GEMMs on the fp8 MFMA (engine.BlockStack,
precision attribute); the text tower (C x 77 rows: too few for the 256x256 fp8 tiles) keeps its
16-bit storage. Tokenisation needs a BPE
tokenizer callable (tokenizer=); without one, set_tokenized_prompts() takes token ids and the
context is initialised from the reference's random branch (maple.py:95-98), or from
ctx_init_tokens (the ids of "a bad photo of a") as its ctx_init branch does.
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn

from . import autograd as lc_autograd
from . import clip_loader
from .adapter_clip import EOT_TOKEN, SOT_TOKEN


def _get_clones(module, N):
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def _tokenize(tokenizer, text, context_length=77):
    ids = [SOT_TOKEN] + list(tokenizer(text)) + [EOT_TOKEN]
    out = torch.zeros(1, context_length, dtype=torch.long)
    ids = ids[:context_length]
    out[0, :len(ids)] = torch.tensor(ids)
    return out


class TextEncoder(nn.Module):
    """maple.py:40-61 (forward on the engine)."""

    def __init__(self, clip_model):
        super().__init__()
        self.transformer = clip_model.transformer
        self.positional_embedding = clip_model.positional_embedding
        self.ln_final = clip_model.ln_final
        self.text_projection = clip_model.text_projection
        self.dtype = clip_model.dtype
        self._clip = [clip_model]  # not a submodule (the reference does not register it)

    def forward(self, prompts, tokenized_prompts, compound_prompts_deeper_text, consumer=None):
        """consumer: the stream that reads the features, when this runs on another one."""
        x0 = prompts + self.positional_embedding
        return lc_autograd.maple_text_apply(self._clip[0].text_tower, tokenized_prompts, x0,
                                            list(compound_prompts_deeper_text), self.training,
                                            consumer=consumer)


class MultiModalPromptLearner(nn.Module):
    """maple.py:64-140."""

    def __init__(self, clip_model, n_ctx=3, tokenizer=None, ctx_init_tokens=None):
        super().__init__()
        self.current_class_names = []
        ctx_init = "a bad photo of a"
        self.dtype = clip_model.dtype
        ctx_dim = clip_model.ln_final.weight.shape[0]
        vis_dim = clip_model.visual.width
        self.compound_prompts_depth = 3
        self.n_ctx = n_ctx
        prompt = None
        if n_ctx <= 4 and tokenizer is not None:
            prompt = _tokenize(tokenizer, ctx_init)
        elif n_ctx <= 4 and ctx_init_tokens is not None:
            prompt = torch.as_tensor(ctx_init_tokens, dtype=torch.long).reshape(1, -1)
        if prompt is not None:  # maple.py:86-93
            w = clip_model.token_embedding.weight
            with torch.no_grad():
                embedding = w.detach()[prompt.to(w.device)]
            ctx_vectors = embedding[0, 1:1 + n_ctx, :].clone()
            self.prompt_prefix = ctx_init
        else:  # maple.py:94-98
            ctx_vectors = torch.empty(n_ctx, ctx_dim)
            nn.init.normal_(ctx_vectors, std=0.02)
            self.prompt_prefix = " ".join(["X"] * n_ctx)
        self.proj = nn.Linear(ctx_dim, vis_dim)
        self.ctx = nn.Parameter(ctx_vectors)
        self.compound_prompts_text = nn.ParameterList([
            nn.Parameter(torch.empty(n_ctx, ctx_dim)) for _ in range(self.compound_prompts_depth - 1)
        ])
        for single_para in self.compound_prompts_text:
            nn.init.normal_(single_para, std=0.02)
        single_layer = nn.Linear(ctx_dim, vis_dim)
        self.compound_prompt_projections = _get_clones(single_layer,
                                                       self.compound_prompts_depth - 1)

    def construct_prompts(self, ctx, prefix, suffix, label=None):
        if label is not None:
            prefix = prefix[label]
            suffix = suffix[label]
        return torch.cat([prefix, ctx, suffix], dim=1)

    def forward(self, prefix, suffix):
        ctx = self.ctx
        if ctx.dim() == 2:
            ctx = ctx.unsqueeze(0).expand(prefix.shape[0], -1, -1)
        prompts = self.construct_prompts(ctx, prefix, suffix)
        visual_deep_prompts = [layer(self.compound_prompts_text[i])
                               for i, layer in enumerate(self.compound_prompt_projections)]
        return prompts, self.proj(self.ctx), self.compound_prompts_text, visual_deep_prompts


class MaPLe(nn.Module):
    """maple.py:143-253."""

    def __init__(self, model_name="ViT-B/16", n_ctx=3, device="cpu", tokenizer=None,
                 ctx_init_tokens=None, arch_overrides=None, clip_model=None, precision="bf16",
                 text_precision="fp16"):
        super().__init__()
        self.device = device
        if clip_model is None:
            clip_model = clip_loader.load(model_name, device=None, jit=False,
                                          design_details={"method": "maple",
                                                          "peft_encoder": "none"},
                                          arch_overrides=arch_overrides)
        for p in clip_model.parameters():
            p.requires_grad = False
        self._tokenizer = tokenizer
        self.prompt_learner = MultiModalPromptLearner(clip_model, n_ctx=n_ctx, tokenizer=tokenizer,
                                                      ctx_init_tokens=ctx_init_tokens)
        self.image_encoder = clip_model.visual
        self.text_encoder = TextEncoder(clip_model)
        self.logit_scale = clip_model.logit_scale
        self.dtype = clip_model.dtype
        self.n_ctx = n_ctx
        self.base_clip_model = clip_model
        self.register_buffer("token_prefix", torch.zeros(0))  # SOS
        self.register_buffer("token_suffix", torch.zeros(0))  # CLS, EOS
        self.tokenized_prompts = None
        self.current_class_names = []
        self.prompt_prefix = self.prompt_learner.prompt_prefix
        self.set_precision(precision)
        self.set_text_precision(text_precision)
        if device is not None and str(device) != "cpu":
            self.to(device)

    def set_precision(self, precision):
        """'bf16' or 'fp8' for the image tower's frozen GEMMs."""
        if precision not in ("bf16", "fp8"):
            raise ValueError("precision must be 'bf16' or 'fp8'")
        self.precision = precision
        self.image_encoder.tower.stack.precision = precision
        return self

    def set_text_precision(self, precision):
        """The text tower's 16-bit storage: 'fp16' (default; IEEE half, the reference's own
        MaPLe backbone dtype, maple_clip/model.py:749-772, 826) or 'bf16'. Its backward runs on
        a per-call power-of-two gradient scale (engine.ScaledGrads) and returns the deep-prompt
        and context-embedding gradients unscaled."""
        dt = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(precision)
        if dt is None:
            raise ValueError("text_precision must be 'fp16' or 'bf16'")
        self.base_clip_model.transformer.engine.set_storage(dt)
        self.text_precision = precision
        return self

    @classmethod
    def from_state_dict(cls, state_dict, n_ctx=3, device=None, precision="bf16", **kwargs):
        from .model import build_model
        bb = build_model(dict(state_dict), {"method": "maple", "peft_encoder": "none"})
        return cls(n_ctx=n_ctx, device=device, clip_model=bb, precision=precision, **kwargs)

    def update_class_names(self, new_class_names):
        """maple.py:178-187 (needs the tokenizer)."""
        num = 0
        for c in new_class_names:
            if c not in self.current_class_names:
                self.current_class_names.append(c)
                num += 1
        if num > 0:
            self.tokenized_prompts, self.token_prefix, self.token_suffix = \
                self.get_tokenized_prompts(self.current_class_names)
        return self.tokenized_prompts

    def get_tokenized_prompts(self, classnames):
        """maple.py:189-206."""
        if self._tokenizer is None:
            raise RuntimeError("no BPE tokenizer configured; use set_tokenized_prompts(ids)")
        classnames = [name.replace("_", " ") for name in classnames]
        prompts = [self.prompt_prefix + " " + name + "." for name in classnames]
        tokenized = torch.cat([_tokenize(self._tokenizer, p) for p in prompts])
        return self._split(tokenized)

    def _split(self, tokenized):
        w = self.base_clip_model.token_embedding.weight
        tokenized = tokenized.to(w.device)
        with torch.no_grad():
            embedding = w.detach()[tokenized]
        return tokenized, embedding[:, :1, :], embedding[:, 1 + self.n_ctx:, :]

    def set_tokenized_prompts(self, tokenized):
        """Token ids [C, 77] of "<prompt_prefix> <class>." (the output of
        get_tokenized_prompts for a tokenizer that runs elsewhere)."""
        self.tokenized_prompts, self.token_prefix, self.token_suffix = self._split(tokenized)
        return self.tokenized_prompts

    def forward(self, image, tokenized_prompts=None, prefix=None, suffix=None):
        """maple.py:208-236: logits = exp(logit_scale) * norm(I) @ norm(T)^T."""
        if tokenized_prompts is None:
            tokenized_prompts = self.tokenized_prompts
            prefix = self.token_prefix
            suffix = self.token_suffix
        vis = self.image_encoder
        side = self._text_stream(image)
        if side is None:
            prompts, shared_ctx, deep_text, deep_vision = self.prompt_learner(prefix, suffix)
            text_features = self.text_encoder(prompts, tokenized_prompts, deep_text)
            image_features = lc_autograd.maple_image_apply(vis.tower, image, shared_ctx,
                                                           deep_vision, self.training)
        else:
            # The towers are independent until the head: the text tower (C prompts x 77 tokens,
            # trained through its deep prompts, so never cached) runs on a side stream beside
            # the image tower, forward and backward (autograd runs each backward on its forward's
            # stream). The text function is applied after the image one so that its backward
            # (the higher sequence number) is launched first and overlaps the image backward.
            # The prompt learner runs on the side stream too: its leaves (ctx, the deep text
            # prompts, the projections) are then read on ONE stream, so their AccumulateGrad
            # nodes and every gradient reaching them live on that stream (r4 read the deep text
            # prompts on both streams: torch warned about the stream mismatch and inserted a
            # cross-stream sync at every accumulation). The image tower waits for the learner's
            # few small launches only.
            main = torch.cuda.current_stream(image.device)
            if self.learner_on_side:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    prompts, shared_ctx, deep_text, deep_vision = self.prompt_learner(prefix, suffix)
                learned = torch.cuda.Event()
                learned.record(side)
                main.wait_event(learned)
                for t in (shared_ctx, *deep_vision):
                    t.record_stream(main)
            else:  # r4: the learner on the main stream (A/Bs)
                prompts, shared_ctx, deep_text, deep_vision = self.prompt_learner(prefix, suffix)
                side.wait_stream(main)
                prompts.record_stream(side)
            image_features = lc_autograd.maple_image_apply(vis.tower, image, shared_ctx,
                                                           deep_vision, self.training)
            with torch.cuda.stream(side):
                text_features = self.text_encoder(prompts, tokenized_prompts, deep_text,
                                                  consumer=main)
            main.wait_stream(side)
        logits, _, _ = lc_autograd.head_apply(image_features, text_features, self.logit_scale,
                                              probs=False)
        return logits

    # the text tower on its own HIP stream beside the image tower (False: one stream, for A/Bs)
    overlap_text = True
    # with overlap_text: the prompt learner on the text stream too (False: r4's main-stream
    # learner, whose deep text prompts were read on both streams; for A/Bs)
    learner_on_side = True

    def _text_stream(self, image):
        if not (self.overlap_text and image.is_cuda):
            return None
        s = getattr(self, "_side", None)
        if s is None or s.device != image.device:
            s = self._side = torch.cuda.Stream(device=image.device)
        return s
