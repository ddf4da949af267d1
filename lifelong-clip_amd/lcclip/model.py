"""torch.nn.Module surface mirroring models/clip/model.py, models/clip/lora.py and
models/clip/adapter.py of qcNPU/LifeLong-CLIP. Parameter names, shapes and initialisation follow
the reference byte-for-byte so its freeze filter (methods/adapter_clip.py:117-119) and the OpenAI
state-dict keys keep working; forward passes run as fused tower kernels (lcclip.engine) instead
of per-op ATen calls.

Deviations from the reference HEAD (all because HEAD cannot run):
  Q1 blocks are called as blk(x) (fixes model.py:780); Q2 PEFT parameters missing from a
  checkpoint keep their init (load_state_dict strict=False); Q3 no hard-coded .cuda().
Only the backbone-frozen training regime is supported: if a backbone parameter requires grad
while autograd is recording, forward raises (the reference freezes it in
online_before_task, methods/adapter_clip.py:115-119).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn

from . import autograd as lc_autograd
from .engine import BlockStack, ImageTower, TextTower


class LayerNorm(nn.LayerNorm):
    """model.py:194-200 (fp32 LayerNorm); parameter container — the kernels read weight/bias."""


class QuickGELU(nn.Module):
    """model.py:203-206; applied inside the fused c_fc GEMM epilogue."""

    def forward(self, x):
        raise RuntimeError("QuickGELU runs fused inside lc_gemm_nt (EPI_GELU)")


class MultiheadAttention(nn.Module):
    """Parameter layout of torch nn.MultiheadAttention(embed_dim, num_heads) with
    _qkv_same_embed_dim (model.py:217): in_proj_weight [3D, D], in_proj_bias [3D], out_proj."""

    def __init__(self, embed_dim: int, num_heads: int):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        if self.head_dim * num_heads != embed_dim:
            raise ValueError("embed_dim must be divisible by num_heads")
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
        self.out_proj = self._make_out_proj(embed_dim)
        self._reset_parameters()

    def _make_out_proj(self, d):
        return nn.Linear(d, d, bias=True)

    def _reset_parameters(self):  # torch MultiheadAttention._reset_parameters
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.constant_(self.in_proj_bias, 0.0)
        nn.init.constant_(self.out_proj.bias, 0.0)


class LoRALinear(nn.Linear):
    """lora.py:100-173 (Linear with r > 0, merge_weights=False): lora_A [r, in] kaiming(a=sqrt5),
    lora_B [out, r] zeros, scaling = alpha / r."""

    def __init__(self, in_features, out_features, r=4, lora_alpha=1, bias=True):
        self.r = r
        self.lora_alpha = lora_alpha
        nn.Linear.__init__(self, in_features, out_features, bias=bias)
        self.lora_A = nn.Parameter(self.weight.new_zeros((r, in_features)))
        self.lora_B = nn.Parameter(self.weight.new_zeros((out_features, r)))
        self.scaling = lora_alpha / r
        self.reset_parameters()

    def reset_parameters(self):
        nn.Linear.reset_parameters(self)
        if hasattr(self, "lora_A"):
            nn.init.kaiming_uniform_(self.lora_A, a=math.sqrt(5))
            nn.init.zeros_(self.lora_B)


class LoRAMultiheadAttention(MultiheadAttention):
    """lora.py:371-452: in_proj_weight_lora_A [r, D] shared by q/k/v, in_proj_weight_lora_B
    [3D, r] (both xavier_uniform, so the in-proj LoRA delta is nonzero at init), out_proj is a
    LoRA Linear; scaling = alpha / r."""

    def __init__(self, embed_dim, num_heads, lora_alpha=1, r=4):
        if r <= 0:
            raise ValueError("r must be > 0")
        self.r = r
        self.lora_alpha = lora_alpha
        self.scaling = lora_alpha / r
        self._lora_ready = False
        super().__init__(embed_dim, num_heads)
        self.in_proj_weight_lora_A = nn.Parameter(torch.empty(r, embed_dim))
        self.in_proj_weight_lora_B = nn.Parameter(torch.empty(3 * embed_dim, r))
        self._lora_ready = True
        self._reset_parameters()

    def _make_out_proj(self, d):
        return LoRALinear(d, d, r=self.r, lora_alpha=self.lora_alpha, bias=True)

    def _reset_parameters(self):
        super()._reset_parameters()
        if getattr(self, "_lora_ready", False):
            nn.init.xavier_uniform_(self.in_proj_weight_lora_A)
            nn.init.xavier_uniform_(self.in_proj_weight_lora_B)


class Adapter(nn.Module):
    """adapter.py:11-72 with init_option='lora', adapter_scalar=0.1, layernorm 'none'
    (model.py:430-437). down_proj width is hard-coded to 64 (adapter.py:38, Q7)."""

    def __init__(self, d_model, bottleneck=64, dropout=0.1, adapter_scalar=0.1):
        super().__init__()
        self.n_embd = d_model
        self.down_size = bottleneck
        self.scale = float(adapter_scalar)
        self.dropout = dropout
        self.down_proj = nn.Linear(d_model, 64)
        self.non_linear_func = nn.ReLU()
        self.up_proj = nn.Linear(bottleneck, d_model)
        if bottleneck != 64:
            raise ValueError("the reference hard-codes the adapter down width to 64 (adapter.py:38)")
        with torch.no_grad():
            nn.init.kaiming_uniform_(self.down_proj.weight, a=math.sqrt(5))
            nn.init.zeros_(self.up_proj.weight)
            nn.init.zeros_(self.down_proj.bias)
            nn.init.zeros_(self.up_proj.bias)


class ResidualAttentionBlock(nn.Module):
    """model.py:209-236."""
    variant = "vanilla"

    def __init__(self, d_model, n_head, attn_mask=None, design_details=None):
        super().__init__()
        self.attn = self._make_attn(d_model, n_head, design_details or {})
        self.ln_1 = LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(d_model, d_model * 4)),
                                              ("gelu", QuickGELU()),
                                              ("c_proj", nn.Linear(d_model * 4, d_model))]))
        self.ln_2 = LayerNorm(d_model)
        self.attn_mask = attn_mask

    def _make_attn(self, d_model, n_head, dd):
        return MultiheadAttention(d_model, n_head)

    def peft_parameters(self):
        return [p for n, p in self.named_parameters() if "lora" in n or "adaptmlp" in n]

    def backbone_parameters(self):
        return [p for n, p in self.named_parameters() if not ("lora" in n or "adaptmlp" in n)]

    def forward(self, x):
        raise RuntimeError("blocks run as a fused stack: call the parent Transformer")


class ResidualAttentionBlock_LoRA(ResidualAttentionBlock):
    """model.py:400-415."""
    variant = "lora"

    def _make_attn(self, d_model, n_head, dd):
        self.lora_alpha = dd.get("lora_alpha", 1)
        self.lora_r = dd.get("lora_r", 4)
        return LoRAMultiheadAttention(d_model, n_head, lora_alpha=self.lora_alpha, r=self.lora_r)


class ResidualAttentionBlock_Adapter(ResidualAttentionBlock):
    """model.py:418-442: one Adapter applied to both sub-block outputs (Q6)."""
    variant = "adapter"

    def __init__(self, d_model, n_head, attn_mask=None, design_details=None):
        super().__init__(d_model, n_head, attn_mask, design_details)
        self.ffn_num = (design_details or {}).get("ffn_num", 64)
        self.adaptmlp = Adapter(d_model=d_model, dropout=0.1, bottleneck=self.ffn_num,
                                adapter_scalar=0.1)


class Transformer(nn.Module):
    """model.py:639-686. forward(x) takes the reference's sequence-first x [L, N, D]."""

    def __init__(self, width, layers, heads, attn_mask=None, design_details=None, modal="text"):
        super().__init__()
        dd = design_details or {}
        self.width = width
        self.layers = layers
        self.heads = heads
        self.causal = attn_mask is not None
        res_type = dd.get("method", "vanilla")
        peft_flag = dd.get("peft_encoder", "none") in ["both", modal]
        if res_type == "adapter" and peft_flag:
            cls = ResidualAttentionBlock_Adapter
        elif res_type == "lora" and peft_flag:
            cls = ResidualAttentionBlock_LoRA
        elif res_type in ("moe", "prefix_prompt") and peft_flag:
            raise NotImplementedError(f"PEFT method {res_type!r} is outside this build's scope "
                                      "(SURVEY.md §2.1)")
        else:
            cls = ResidualAttentionBlock
        self.resblocks = nn.Sequential(*[cls(width, heads, attn_mask, dd) for _ in range(layers)])
        self.variant = cls.variant
        self._engine = None

    @property
    def engine(self) -> BlockStack:
        if self._engine is None:
            self._engine = BlockStack(list(self.resblocks), self.heads, self.causal, self.variant)
        return self._engine

    def forward(self, x):
        L, N, D = x.shape
        x2 = x.permute(1, 0, 2).reshape(N * L, D).contiguous().float()
        y = lc_autograd.stack_apply(self, x2, N, L)
        return y.reshape(N, L, D).permute(1, 0, 2)


class VisualTransformer(nn.Module):
    """model.py:689-787."""

    def __init__(self, input_resolution, patch_size, width, layers, heads, output_dim, modal=None,
                 design_details=None):
        super().__init__()
        self.input_resolution = input_resolution
        self.output_dim = output_dim
        self.patch_size = patch_size
        self.width = width
        self.layers = layers
        self.heads = heads
        self.conv1 = nn.Conv2d(in_channels=3, out_channels=width, kernel_size=patch_size,
                               stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(
            scale * torch.randn((input_resolution // patch_size) ** 2 + 1, width))
        self.ln_pre = LayerNorm(width)
        self.transformer = Transformer(width, layers, heads, modal=modal,
                                       design_details=design_details)
        self.ln_post = LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))
        self._tower = None

    @property
    def tower(self) -> ImageTower:
        if self._tower is None:
            self._tower = ImageTower(self, self.transformer.engine)
        return self._tower

    def forward(self, x):
        return lc_autograd.tower_apply(self.tower, self.transformer, x, self.training)


class CLIP(nn.Module):
    """model.py:790-975 (ViT visual tower only; ModifiedResNet is out of scope)."""

    def __init__(self, embed_dim, image_resolution, vision_layers, vision_width,
                 vision_patch_size, context_length, vocab_size, transformer_width,
                 transformer_heads, transformer_layers, design_details):
        super().__init__()
        self.design_details = design_details
        self.context_length = context_length
        if isinstance(vision_layers, (tuple, list)):
            raise NotImplementedError("ModifiedResNet visual towers are out of scope (SURVEY.md §2.1)")
        vision_heads = vision_width // 64
        self.visual = VisualTransformer(input_resolution=image_resolution,
                                        patch_size=vision_patch_size, width=vision_width,
                                        layers=vision_layers, heads=vision_heads,
                                        output_dim=embed_dim, modal="image",
                                        design_details=design_details)
        self.transformer = Transformer(width=transformer_width, layers=transformer_layers,
                                       heads=transformer_heads,
                                       attn_mask=self.build_attention_mask(), modal="text",
                                       design_details=design_details)
        self.vocab_size = vocab_size
        self.token_embedding = nn.Embedding(vocab_size, transformer_width)
        self.positional_embedding = nn.Parameter(torch.empty(self.context_length, transformer_width))
        self.ln_final = LayerNorm(transformer_width)
        self.text_projection = nn.Parameter(torch.empty(transformer_width, embed_dim))
        self.logit_scale = nn.Parameter(torch.ones([]) * np.log(1 / 0.07))
        self.initialize_parameters()
        self._text_tower = None

    def initialize_parameters(self):
        """model.py:852-885 (text blocks only, as in the reference)."""
        nn.init.normal_(self.token_embedding.weight, std=0.02)
        nn.init.normal_(self.positional_embedding, std=0.01)
        with torch.no_grad():
            self.logit_scale.fill_(float(np.log(1 / 0.07)))
        proj_std = (self.transformer.width ** -0.5) * ((2 * self.transformer.layers) ** -0.5)
        attn_std = self.transformer.width ** -0.5
        fc_std = (2 * self.transformer.width) ** -0.5
        for block in self.transformer.resblocks:
            nn.init.normal_(block.attn.in_proj_weight, std=attn_std)
            nn.init.normal_(block.attn.out_proj.weight, std=proj_std)
            nn.init.normal_(block.mlp.c_fc.weight, std=fc_std)
            nn.init.normal_(block.mlp.c_proj.weight, std=proj_std)
        if self.text_projection is not None:
            nn.init.normal_(self.text_projection, std=self.transformer.width ** -0.5)

    def build_attention_mask(self):
        """model.py:926-932: additive causal mask (-inf above the diagonal)."""
        mask = torch.empty(self.context_length, self.context_length)
        mask.fill_(float("-inf"))
        mask.triu_(1)
        return mask

    @property
    def dtype(self):
        return self.visual.conv1.weight.dtype

    @property
    def text_tower(self) -> TextTower:
        if self._text_tower is None:
            self._text_tower = TextTower(self, self.transformer.engine)
        return self._text_tower

    def encode_image(self, image):
        # model.py:938-939 casts the image batch to the model dtype; a 2-D input is conv1's bf16
        # patch rows from the fused train transform and is passed through as is
        return self.visual(image if image.dim() == 2 else image.type(self.dtype))

    def encode_text(self, text):
        return lc_autograd.tower_apply(self.text_tower, self.transformer, text, self.training)

    def forward(self, image, text):
        if image is None:
            return self.encode_text(text)
        elif text is None:
            return self.encode_image(image)
        image_features = self.encode_image(image)
        text_features = self.encode_text(text)
        logits_per_image, image_features, text_features = lc_autograd.head_apply(
            image_features, text_features, self.logit_scale, probs=False)
        return logits_per_image, logits_per_image.t(), image_features, text_features


def build_model(state_dict: dict, design_details: dict):
    """model.py:1005-1062 shape inference; loads with strict=False (Q2) and keeps fp32."""
    if "visual.proj" not in state_dict:
        raise NotImplementedError("only ViT CLIP checkpoints are supported")
    vision_width = state_dict["visual.conv1.weight"].shape[0]
    vision_layers = len([k for k in state_dict.keys()
                         if k.startswith("visual.") and k.endswith(".attn.in_proj_weight")])
    vision_patch_size = state_dict["visual.conv1.weight"].shape[-1]
    grid_size = round((state_dict["visual.positional_embedding"].shape[0] - 1) ** 0.5)
    image_resolution = vision_patch_size * grid_size
    embed_dim = state_dict["text_projection"].shape[1]
    context_length = state_dict["positional_embedding"].shape[0]
    vocab_size = state_dict["token_embedding.weight"].shape[0]
    transformer_width = state_dict["ln_final.weight"].shape[0]
    transformer_heads = transformer_width // 64
    transformer_layers = len(set(k.split(".")[2] for k in state_dict
                                 if k.startswith("transformer.resblocks")))
    model = CLIP(embed_dim, image_resolution, vision_layers, vision_width, vision_patch_size,
                 context_length, vocab_size, transformer_width, transformer_heads,
                 transformer_layers, design_details)
    sd = {k: v for k, v in state_dict.items()
          if k not in ("input_resolution", "context_length", "vocab_size")}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    # strict=False semantics restricted to PEFT tensors (Q2): backbone keys must match exactly
    bad_missing = [k for k in missing if "lora" not in k and "adaptmlp" not in k]
    bad_unexp = [k for k in unexpected if "lora" not in k and "adaptmlp" not in k]
    if bad_missing or bad_unexp:
        raise RuntimeError(f"state dict mismatch: missing {bad_missing[:5]}, unexpected {bad_unexp[:5]}")
    for p in model.parameters():
        p.data = p.data.float()
    return model.eval()
