"""CLIP_MVP — drop-in for models/mvp_clip.py:17-297 of qcNPU/LifeLong-CLIP (BASELINE config 3:
MVP, mask + visual prompt, frozen backbone).

Same constructor arguments, parameters (key, mask, g_prompts, e_prompts), buffers (pos_g_prompt,
pos_e_prompt, similarity, count), attributes (backbone, features, similarity_loss, text_tokens,
current_class_names, prompt_template) and methods (labels_tokenize, set_exposed_classes,
prompt_tuning, forward_features -> (x, text_features, mask), forward_head, forward, loss_fn,
get_similarity_loss). The image work runs on the liblcclip engine: one embed (conv1 + CLS/pos +
ln_pre), the no-grad key query over the first 11 or 12 blocks, and the prompt-tuned pass whose
blocks run at L + P where prompts are appended (197 -> 202 at the g-prompt layers, 217 at the
e-prompt layers); backward returns the gradients of the appended prompt rows. The text tower is
frozen here (peft_encoder 'none'), so its features are cached per token tensor
instead of being recomputed every step as the reference does.

Selection, key distance, mask and the small [B, pool] / [B, C] tensors stay torch ops, as in the
reference.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import autograd as lc_autograd
from . import clip_loader
from .adapter_clip import EOT_TOKEN, SOT_TOKEN
from .textcache import TokenFeatureCache


class _PoolGather(torch.autograd.Function):
    """table[idx] for a small pool (the selected e-prompts / masks, mvp_clip.py:236-237): the same
    gather forward; the backward sums each selected row's gradient into its pool entry as one
    GEMM (one_hot(idx)^T @ grad) instead of torch's sort-based index_put accumulate, which
    serialises the 128 images that pick the same few entries (0.39 ms per config-3 step)."""

    @staticmethod
    def forward(ctx, table, idx):
        ctx.save_for_backward(idx)
        ctx.pool = table.shape[0]
        return table[idx]

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        flat = idx.reshape(-1)
        onehot = F.one_hot(flat, ctx.pool).to(g.dtype)
        gt = onehot.t() @ g.reshape(flat.numel(), -1)
        return gt.reshape(ctx.pool, *g.shape[idx.dim():]), None


# LCCLIP_POOL_GEMM=0: plain indexing (torch's index_put backward), for A/Bs
_POOL_GEMM = os.environ.get("LCCLIP_POOL_GEMM", "1") != "0"


def _pool_gather(table, idx):
    return _PoolGather.apply(table, idx) if _POOL_GEMM else table[idx]


class CLIP_MVP(nn.Module):
    def __init__(self, pos_g_prompt: Iterable[int] = (0, 1), len_g_prompt: int = 5,
                 pos_e_prompt: Iterable[int] = (2, 3, 4), len_e_prompt: int = 20,
                 selection_size: int = 1, prompt_func: str = "prompt_tuning", task_num: int = 10,
                 num_classes: int = 100, lambd: float = 1.0, use_mask: bool = True,
                 use_contrastiv: bool = False, use_last_layer: bool = True,
                 model_name="ViT-B/16", device="cpu", tokenizer=None, arch_overrides=None,
                 backbone=None, text_precision="fp16", **kwargs):
        super().__init__()
        self.features = torch.empty(0)
        self.keys = torch.empty(0)
        self.lambd = lambd
        self.class_num = num_classes
        self.task_num = task_num
        self.use_mask = use_mask
        self.use_contrastiv = use_contrastiv
        self.use_last_layer = use_last_layer
        self.selection_size = selection_size
        self.device = device
        # mvp_clip.py:51-60: frozen CLIP, vanilla blocks (method 'mvp', peft_encoder 'none')
        if backbone is None:
            backbone = clip_loader.load(model_name, device=None, jit=False,
                                        design_details={"method": "mvp", "peft_encoder": "none"},
                                        arch_overrides=arch_overrides)
        model = backbone
        self.add_module("backbone", model)
        for param in self.backbone.parameters():
            param.requires_grad = False
        self.prompt_template = "a bad photo of a {}."
        self.text_tokens = None
        self.current_class_names = []
        self._tokenizer = tokenizer
        embed_dim = self.backbone.visual.conv1.weight.shape[0]
        # mvp_clip.py:68-104
        self.register_buffer("pos_g_prompt", torch.tensor(pos_g_prompt, dtype=torch.int64))
        self.register_buffer("pos_e_prompt", torch.tensor(pos_e_prompt, dtype=torch.int64))
        self.register_buffer("similarity", torch.zeros(1))
        self.len_g_prompt = len_g_prompt
        self.len_e_prompt = len_e_prompt
        self.g_length = len(pos_g_prompt) if pos_g_prompt else 0
        self.e_length = len(pos_e_prompt) if pos_e_prompt else 0
        g_pool = 1
        e_pool = task_num
        self.register_buffer("count", torch.zeros(e_pool))
        self.key = nn.Parameter(torch.randn(e_pool, embed_dim))
        self.mask = nn.Parameter(torch.zeros(e_pool, self.class_num) - 1)
        if prompt_func == "prompt_tuning":
            self.prompt_func = self.prompt_tuning
            self.g_size = 1 * self.g_length * self.len_g_prompt
            self.e_size = 1 * self.e_length * self.len_e_prompt
        elif prompt_func == "prefix_tuning":
            self.prompt_func = self.prefix_tuning
            self.g_size = 2 * self.g_length * self.len_g_prompt
            self.e_size = 2 * self.e_length * self.len_e_prompt
        else:
            raise ValueError(f"unknown prompt_func {prompt_func!r}")
        self.g_prompts = nn.Parameter(torch.randn(g_pool, self.g_size, embed_dim))
        self.e_prompts = nn.Parameter(torch.randn(e_pool, self.e_size, embed_dim))
        self.exposed_classes = 0
        self._txt_cache = TokenFeatureCache()
        # the frozen text tower's 16-bit storage: IEEE half, the reference's autocast dtype
        # ('bf16' optional); forward only, its features cached
        dt = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(text_precision)
        if dt is None:
            raise ValueError("text_precision must be 'fp16' or 'bf16'")
        self.backbone.transformer.engine.set_storage(dt)
        self.text_precision = text_precision
        if device is not None and str(device) != "cpu":
            self.to(device)

    @classmethod
    def from_state_dict(cls, state_dict, device=None, **kwargs):
        """Build around an in-memory CLIP state dict (clip_loader.py:116-135's local-file path)."""
        from .model import build_model
        bb = build_model(dict(state_dict), {"method": "mvp", "peft_encoder": "none"})
        return cls(backbone=bb, device=device, **kwargs)

    # ------------------------------------------------------------------ text side
    def labels_tokenize(self, labels: Union[str, List[str]], context_length: int = 77):
        """mvp_clip.py:108-140 (needs a BPE tokenizer callable: text -> ids without SOT/EOT)."""
        if self._tokenizer is None:
            raise RuntimeError("no BPE tokenizer configured; pass tokenizer= or token ids")
        if isinstance(labels, str):
            labels = [labels]
        texts = [self.prompt_template.format(c) for c in labels]
        all_tokens = [[SOT_TOKEN] + list(self._tokenizer(t)) + [EOT_TOKEN] for t in texts]
        result = torch.zeros(len(all_tokens), context_length, dtype=torch.long)
        for i, tokens in enumerate(all_tokens):
            tokens = tokens[:context_length]
            result[i, :len(tokens)] = torch.tensor(tokens)
        return result.to(self.key.device)

    @torch.no_grad()
    def set_exposed_classes(self, classes_names):
        """mvp_clip.py:142-156."""
        self.exposed_classes = len(classes_names)
        new = False
        for c in classes_names:
            if c not in self.current_class_names:
                self.current_class_names.append(c)
                new = True
        if new:
            self.text_tokens = self.labels_tokenize(self.current_class_names)
        self.text_tokens = self.text_tokens.to(self.key.device)
        return self.text_tokens

    def encode_text_cached(self, text_tokens):
        """backbone.encode_text (mvp_clip.py:192) for the frozen text tower, cached on the token
        content and the text weights' versions (lcclip.textcache)."""
        tt = self.backbone
        key = (tuple(p._version for p in tt.transformer.parameters()),
               tt.token_embedding.weight._version, tt.text_projection._version,
               tt.ln_final.weight._version)
        f = self._txt_cache.get(text_tokens, key)
        if f is None:
            with torch.no_grad():
                f = tt.encode_text(text_tokens)
            self._txt_cache.put(text_tokens, key, f)
        return f

    # ------------------------------------------------------------------ image side
    def _prompt_layers(self, g_prompt, e_prompt):
        """{layer: [B, P, C]}: the g then e prompt tokens mvp_clip.py:161-172 appends there."""
        B = g_prompt.shape[0] if g_prompt.dim() == 3 else e_prompt.shape[0]
        C = self.backbone.visual.width
        out = {}
        g = g_prompt.contiguous().view(B, -1, self.len_g_prompt, C) if self.g_size else None
        e = e_prompt.contiguous().view(B, -1, self.len_e_prompt, C) if self.e_size else None
        for n in range(self.backbone.visual.layers):
            parts = []
            pos_g = (self.pos_g_prompt == n).nonzero().flatten()
            if g is not None and pos_g.numel():
                parts.append(g[:, pos_g].reshape(B, -1, C))
            pos_e = (self.pos_e_prompt == n).nonzero().flatten()
            if e is not None and pos_e.numel():
                parts.append(e[:, pos_e].reshape(B, -1, C))
            if parts:
                out[n] = torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]
        return out

    def prompt_tuning(self, x0, g_prompt, e_prompt, n=None, L=None, **kwargs):
        """mvp_clip.py:158-175 + ln_post/proj (:259-261) on the engine. x0: embed() output."""
        vis = self.backbone.visual
        return lc_autograd.prompt_tower_apply(vis.tower, vis.transformer, x0, n, L,
                                              self._prompt_layers(g_prompt, e_prompt),
                                              self.training)

    def prefix_tuning(self, x, g_prompt, e_prompt, **kwargs):
        raise NotImplementedError("prefix_tuning not implemented yet")  # mvp_clip.py:177-180

    def forward_features(self, inputs, text_tokens=None, **kwargs):
        """mvp_clip.py:182-264 -> (image features [B, E], text features [C, E], mask [B, C])."""
        self.backbone.visual.eval()
        if text_tokens is None:
            text_tokens = self.text_tokens
        text_features = self.encode_text_cached(text_tokens)
        vis = self.backbone.visual
        tower = vis.tower
        with torch.no_grad():
            x0, n, L, first = tower.embed_query(inputs)
            stop = vis.layers if self.use_last_layer else vis.layers - 1
            query = tower.query(x0, n, L, stop, first_ln1=first)
        B = n
        if self.training:
            self.features = torch.cat((self.features, query.detach().cpu()), dim=0)
        distance = 1 - F.cosine_similarity(query.unsqueeze(1), self.key, dim=-1)
        mass = (self.count + 1) if self.use_contrastiv else 1.0
        scaled_distance = distance * mass
        topk = scaled_distance.topk(self.selection_size, dim=1, largest=False)[1]
        distance = distance[torch.arange(topk.size(0), device=topk.device).unsqueeze(1).repeat(
            1, self.selection_size), topk].squeeze().clone()
        e_prompts = _pool_gather(self.e_prompts, topk).squeeze().clone()
        mask = _pool_gather(self.mask, topk).mean(1).squeeze().clone()
        if self.use_contrastiv:
            key_wise_distance = 1 - F.cosine_similarity(self.key.unsqueeze(1), self.key, dim=-1)
            self.similarity_loss = -((key_wise_distance[topk] / mass[topk]).exp().mean() /
                                     ((distance / mass[topk]).exp().mean() +
                                      (key_wise_distance[topk] / mass[topk]).exp().mean()) +
                                     1e-6).log()
        else:
            self.similarity_loss = distance.mean()
        g_prompts = self.g_prompts[0].repeat(B, 1, 1)
        if self.training:
            with torch.no_grad():
                num = topk.view(-1).bincount(minlength=self.e_prompts.size(0))
                dp = getattr(self, "_dp", None)
                if dp is not None:  # one rank per GPU: count the global batch on every replica
                    dp.all_sum(num)
                self.count += num
        if e_prompts.dim() == 2:  # B == 1: the reference's squeeze() dropped the batch axis
            e_prompts = e_prompts.unsqueeze(0)
        x = self.prompt_func(x0, g_prompts.float(), e_prompts.float(), n=n, L=L)
        mask = torch.sigmoid(mask) * 2.0
        C = (self.text_tokens if self.text_tokens is not None else text_tokens).shape[0]
        return x, text_features, mask[..., :C]

    def forward_head(self, image_features, text_features=None, **kwargs):
        """mvp_clip.py:266-280: cosine logits scaled by exp(logit_scale)."""
        logits, _, _ = lc_autograd.head_apply(image_features, text_features,
                                              self.backbone.logit_scale, probs=False)
        return logits

    def forward(self, inputs, text_tokens=None, **kwargs):
        """mvp_clip.py:282-288."""
        x, text_features, mask = self.forward_features(inputs, text_tokens, **kwargs)
        x = self.forward_head(x, text_features, **kwargs)
        if self.use_mask:
            x = x * mask
        return x

    def loss_fn(self, output, target):
        """mvp_clip.py:290-291."""
        return F.cross_entropy(output, target) + self.similarity_loss

    def get_similarity_loss(self):
        return self.similarity_loss
