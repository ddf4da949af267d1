"""CPU oracle for the CLIP dual-encoder PEFT training step — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product. Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it. The shipped path
(``lifelong-clip_amd/lcclip``) never imports anything under ``oracle/`` and fails loudly
when its HIP library is missing.

What it restates (reference = qcNPU/LifeLong-CLIP @ 2024-12-18; citations are
``path:line`` into that tree, which is read as text only — importing or running it was
refused by the environment, see SURVEY.md §8(c) and DESIGN.md §Oracle):

  * ``layer_norm``            models/clip/model.py:194-200   (fp32 upcast, eps 1e-5)
  * ``quick_gelu``            models/clip/model.py:203-206   (x * sigmoid(1.702 x))
  * ``mha``                   models/clip/lora.py:832-1074   (LoRA in-proj: shared A,
                              stacked B, scaling alpha/r; q *= d_h^-0.5; bmm/softmax/bmm;
                              out-proj + LoRA) and torch nn.MultiheadAttention for the
                              vanilla/adapter blocks (model.py:217, 226-231)
  * ``adapter``               models/clip/adapter.py:53-72   (down 64, ReLU, dropout,
                              up, *scale, + residual; layernorm option 'none')
  * ``block``                 models/clip/model.py:233-236 (vanilla / LoRA) and :439-442
                              (adapter: the SAME adapter applied to both sub-blocks)
  * ``encode_image``          models/clip/model.py:755-787   (Q1: ``blk(x)``, fixing :780)
  * ``encode_text``           models/clip/model.py:941-956 + mask :926-932
  * ``clip_logits``           models/clip/model.py:958-975
  * ``adapter_clip_forward``  models/adapter_clip.py:94-100  (returns softmax probs)
  * ``loss_on_probs``         methods/adapter_clip.py:88-89 + methods/_trainer.py:164
                              (CrossEntropyLoss applied to the probabilities — Q5)
  * ``adamw_step``            utils/train_utils.py:27-28 (torch.optim.AdamW, wd 1e-5)
  * ``mvp_forward``           models/mvp_clip.py:158-291   (CLIP_MVP: no-grad key query,
                              top-1 e-prompt / mask selection, prompt tuning with tokens
                              appended per layer and dropped after it, masked logits)
  * ``maple_forward``         models/maple.py:40-251 + models/maple_clip/model.py:316-401,
                              551-590 (MaPLe: learned text context, shared visual context
                              before ln_pre, deep prompts replacing rows at layers 1..2)

Parity pinning. The reference ships no tests, fixtures or golden vectors and could not be
executed here, so the numeric restatement is pinned by the
reference's own known answers and structural identities (tests/test_oracle.py):
ViT-L/14 adapter-CLIP total/trainable parameter counts from nohup.out:8,29; the
adapter-at-init == vanilla identity (adapter.py:49-51); out-proj LoRA B = 0 at init
(lora.py:133-139); the vanilla block == torch's own nn.MultiheadAttention composition; and
the double-softmax loss band. Golden fixtures under tests/golden/ are generated from this
module by tests/golden/make_golden.py.

Rounding hook. Every function takes ``rt`` (default identity). With ``rt = round_bf16`` the
oracle rounds exactly where the MI355X path rounds (GEMM/attention operands and the bf16
activations it stores), so the HIP forward can be checked at a tight tolerance; with the
identity it is the plain fp32 reference algorithm. ``round_bf16`` / ``round_f16`` are straight-through
(forward rounding only); ``round_bf16_fwd_bwd`` / ``round_f16_fwd_bwd`` (``Rounding``) also round
where the HIP backward stores 16-bit gradients, so the GPU's gradients can be checked against an
oracle that makes the same roundings (its distance then measures implementation error, not
emulation gaps). The MI355X path stores the image tower in bf16 and the text tower in IEEE half
(``rt_text``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

EOT_TOKEN = 49407
SOT_TOKEN = 49406


def identity(x):
    return x


def round_bf16(x):
    """Round-to-nearest-even fp32 -> bf16 -> fp32 (value-preserving forward, STE backward)."""
    r = x.detach().to(torch.bfloat16).to(x.dtype)
    return x + (r - x).detach()


def _bf(x):
    return x.to(torch.bfloat16).to(x.dtype)


def _hf(x):
    return x.to(torch.float16).to(x.dtype)


def round_f16(x):
    """Round-to-nearest-even fp32 -> IEEE half -> fp32 (value-preserving forward, STE backward):
    the MI355X text tower's storage (lcclip AdapterCLIP text_precision='fp16', the reference's
    autocast dtype, methods/adapter_clip.py:87)."""
    r = _hf(x.detach())
    return x + (r - x).detach()


# The MI355X image towers keep the residual stream in IEEE half, the reference's autocast dtype
# (model.py:194-200: its LayerNorm returns the input dtype, so x is fp16 from conv1 through every
# `x = x + ...`; lcclip ImageTower.RESID16, widths 512 / 768): encode_image / mvp_forward /
# maple_forward round x there with the image rounding's ``resid`` hook. round_f16 is
# straight-through; the backward-faithful ``Rounding.resid`` also rounds the residual gradient
# under the per-call scale (the adapter and LoRA towers' half gradient; the frozen prompt towers
# keep an f32 gradient on the GPU).
round_bf16.resid = round_f16


class _GradRound(torch.autograd.Function):
    """Identity forward; the incoming gradient rounded by `rnd`: a point where the HIP backward
    stores a 16-bit gradient that the next GEMM reads."""

    @staticmethod
    def forward(ctx, x, rnd):
        ctx.rnd = rnd
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return ctx.rnd(g), None


class _GradScaleSet(torch.autograd.Function):
    """Identity forward; in backward sets the hook's gradient scale from the incoming gradient,
    s = 2^(e - floor(log2 max|g|)) (the per-call loss scale of the IEEE-half text tower, e = 10,
    and of the image tower's half residual gradient, e = 12: ops.grad_pow2_normalize /
    head.hip), before any rounding inside the tower runs."""

    @staticmethod
    def forward(ctx, x, hook, e=10):
        ctx.hook, ctx.e = hook, e
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        a = g.abs().max().item()
        ctx.hook.gs = 2.0 ** (ctx.e - math.floor(math.log2(a))) if 0 < a < float("inf") else 1.0
        return g, None, None


class _ResidRound(torch.autograd.Function):
    """The half residual stream of the MI355X image tower (ImageTower.RESID16): x rounded to
    IEEE half; its gradient stored in half too, carrying the hook's power-of-two scale gs
    (lcclip ImageTower.backward: ops.grad_pow2_normalize, target 2^12; lc_layernorm_bwd_g16)."""

    @staticmethod
    def forward(ctx, x, hook):
        ctx.hook = hook
        return _hf(x)

    @staticmethod
    def backward(ctx, g):
        s = ctx.hook.gs
        return _hf(g * s) / s, None


class _QuickGeluRound(torch.autograd.Function):
    """quick_gelu whose backward multiplies by QuickGELU'(pre) rounded to the storage type: the
    c_fc epilogue stores the derivative (EPI_GELU_D, gemm.hip) and the c_proj input-gradient
    epilogue multiplies its f32 accumulator by it (EPI_MUL); the product is rounded where the
    caller puts the gradient rounding."""

    @staticmethod
    def forward(ctx, x, rnd):
        ctx.save_for_backward(x)
        ctx.rnd = rnd
        return quick_gelu(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        sg = torch.sigmoid(1.702 * x)
        return g * ctx.rnd(sg + 1.702 * x * sg * (1 - sg)), None


class _AttnCoreRound(torch.autograd.Function):
    """attention_core's rounded forward, with the backward of the HIP kernel
    (attention.hip:456-806) on the 16-bit q, k, v, O, dO: P = exp(S - lse) recomputed in f32,
    D = rowsum(dO O), dS = P (dO V^T - D); dV = P_16^T dO, dK = scale dS_16^T Q,
    dQ = scale dS_16 K, each stored 16-bit. rnd rounds values (P), grnd gradients (dO, dS and
    the dq|dk|dv store; the IEEE-half tower's carry its loss scale)."""

    @staticmethod
    def forward(ctx, q, k, v, scale, causal, rnd, grnd):
        s = (q @ k.transpose(-1, -2)) * scale
        if causal:
            L = s.shape[-1]
            s = s + torch.full((L, L), float("-inf")).triu_(1)
        m = s.amax(dim=-1, keepdim=True)
        pe = torch.exp(s - m)
        l = pe.sum(dim=-1, keepdim=True)
        o = rnd((rnd(pe) @ v) / l)
        ctx.save_for_backward(q, k, v, o, m + torch.log(l))
        ctx.scale, ctx.causal, ctx.rnd, ctx.grnd = scale, causal, rnd, grnd
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        scale, rnd, grnd = ctx.scale, ctx.rnd, ctx.grnd
        do = grnd(do)
        s = (q @ k.transpose(-1, -2)) * scale
        if ctx.causal:
            L = s.shape[-1]
            s = s + torch.full((L, L), float("-inf")).triu_(1)
        p = torch.exp(s - lse)
        d = (do * o).sum(dim=-1, keepdim=True)
        ds = p * (do @ v.transpose(-1, -2) - d)
        dsb = grnd(ds)
        dq = grnd(scale * (dsb @ k))
        dk = grnd(scale * (dsb.transpose(-1, -2) @ q))
        dv = grnd(rnd(p).transpose(-1, -2) @ do)
        return dq, dk, dv, None, None, None, None


class Rounding:
    """A rounding hook for the oracle's ``rt`` argument: called on a tensor it rounds the value
    to the storage type (straight-through gradient), like ``round_bf16``. With backward=True it
    also carries the HIP backward's roundings, read by the functions that take ``rt``:
    ``bwd`` (the gradient rounding at each 16-bit gradient store: the features' gradient, dY
    into each input-gradient GEMM, dpre, dz, da, dh, dO), ``gelu`` (the stored QuickGELU') and
    ``attn`` (the attention backward above); kind 'f16' adds ``top`` (the per-call gradient
    scale, set at the tower output and applied inside every gradient rounding)."""

    def __init__(self, kind, backward=False):
        self.kind = kind
        self._rnd = {"bf16": _bf, "f16": _hf}[kind]
        self.gs = 1.0
        if kind == "bf16":
            self.resid = round_f16  # the image tower's half residual stream (round_bf16.resid)
        if backward:
            self.bwd = lambda x: _GradRound.apply(x, self._grnd)
            self.gelu = lambda x: _QuickGeluRound.apply(x, self._rnd)
            self.attn = lambda q, k, v, scale, causal: _AttnCoreRound.apply(
                q, k, v, scale, causal, self._rnd, self._grnd)
            if kind == "f16":
                self.top = lambda x: _GradScaleSet.apply(x, self)
            else:  # the image tower: its half residual gradient's scale (bf16 roundings ignore it)
                self.top = lambda x: _GradScaleSet.apply(x, self, 12)
                self.resid = lambda x: _ResidRound.apply(x, self)

    def __call__(self, x):
        r = self._rnd(x.detach())
        return x + (r - x).detach()

    def _grnd(self, g):
        s = self.gs
        return self._rnd(g * s) / s if s != 1.0 else self._rnd(g)


# forward + backward roundings of the MI355X path: the image tower (bf16) and the text tower
# (IEEE half, text_precision='fp16'); the straight-through round_bf16 / round_f16 round the
# forward only, so their gradients miss the backward's roundings
round_bf16_fwd_bwd = Rounding("bf16", backward=True)
round_f16_fwd_bwd = Rounding("f16", backward=True)


@dataclass(frozen=True)
class ClipConfig:
    """CLIP shape parameters, inferred the way build_model does (model.py:1005-1049)."""
    embed_dim: int = 512
    image_resolution: int = 224
    vision_layers: int = 12
    vision_width: int = 768
    vision_patch_size: int = 16
    context_length: int = 77
    vocab_size: int = 49408
    transformer_width: int = 512
    transformer_heads: int = 8
    transformer_layers: int = 12

    @property
    def vision_heads(self):  # model.py:820
        return self.vision_width // 64

    @property
    def grid(self):
        return self.image_resolution // self.vision_patch_size


VIT_B16 = ClipConfig()
VIT_L14 = ClipConfig(embed_dim=768, vision_layers=24, vision_width=1024, vision_patch_size=14,
                     transformer_width=768, transformer_heads=12)


def tower_prefixes(cfg: ClipConfig):
    vis = [f"visual.transformer.resblocks.{i}." for i in range(cfg.vision_layers)]
    txt = [f"transformer.resblocks.{i}." for i in range(cfg.transformer_layers)]
    return vis, txt


def peft_on(peft_encoder: str, modal: str) -> bool:
    """model.py:653-654: PEFT blocks are used when peft_encoder in ['both', modal]."""
    return peft_encoder in ("both", modal)


# ----------------------------------------------------------------------------- parameters
def param_shapes(cfg: ClipConfig, method: str = "vanilla", peft_encoder: str = "none",
                 lora_r: int = 4, ffn_num: int = 64):
    """Name -> shape, in the reference's named_parameters() naming.

    Backbone: model.py:709-729 (visual), 830-845 (text), 209-223 (blocks).
    LoRA: lora.py:419-422 (in_proj_weight_lora_A [r, D], _B [3D, r]), lora.py:123-125
    (out_proj.lora_A [r, D], lora_B [D, r]). Adapter: adapter.py:38-40 (down width is the
    hard-coded 64, Q7). Block placement: model.py:652-683.
    """
    s = {}
    W, P, E = cfg.vision_width, cfg.vision_patch_size, cfg.embed_dim
    s["visual.class_embedding"] = (W,)
    s["visual.positional_embedding"] = (cfg.grid ** 2 + 1, W)
    s["visual.proj"] = (W, E)
    s["visual.conv1.weight"] = (W, 3, P, P)
    s["visual.ln_pre.weight"] = (W,)
    s["visual.ln_pre.bias"] = (W,)
    s["visual.ln_post.weight"] = (W,)
    s["visual.ln_post.bias"] = (W,)
    T = cfg.transformer_width
    s["positional_embedding"] = (cfg.context_length, T)
    s["text_projection"] = (T, E)
    s["logit_scale"] = ()
    s["token_embedding.weight"] = (cfg.vocab_size, T)
    s["ln_final.weight"] = (T,)
    s["ln_final.bias"] = (T,)
    vis, txt = tower_prefixes(cfg)
    for modal, width, prefixes in (("image", W, vis), ("text", T, txt)):
        use = peft_on(peft_encoder, modal)
        for pre in prefixes:
            s[pre + "attn.in_proj_weight"] = (3 * width, width)
            s[pre + "attn.in_proj_bias"] = (3 * width,)
            if use and method == "lora":
                s[pre + "attn.in_proj_weight_lora_A"] = (lora_r, width)
                s[pre + "attn.in_proj_weight_lora_B"] = (3 * width, lora_r)
            s[pre + "attn.out_proj.weight"] = (width, width)
            s[pre + "attn.out_proj.bias"] = (width,)
            if use and method == "lora":
                s[pre + "attn.out_proj.lora_A"] = (lora_r, width)
                s[pre + "attn.out_proj.lora_B"] = (width, lora_r)
            s[pre + "ln_1.weight"] = (width,)
            s[pre + "ln_1.bias"] = (width,)
            s[pre + "mlp.c_fc.weight"] = (4 * width, width)
            s[pre + "mlp.c_fc.bias"] = (4 * width,)
            s[pre + "mlp.c_proj.weight"] = (width, 4 * width)
            s[pre + "mlp.c_proj.bias"] = (width,)
            s[pre + "ln_2.weight"] = (width,)
            s[pre + "ln_2.bias"] = (width,)
            if use and method == "adapter":
                s[pre + "adaptmlp.down_proj.weight"] = (64, width)
                s[pre + "adaptmlp.down_proj.bias"] = (64,)
                s[pre + "adaptmlp.up_proj.weight"] = (width, ffn_num)
                s[pre + "adaptmlp.up_proj.bias"] = (width,)
    return s


def is_trainable(name: str) -> bool:
    """Freeze filter, methods/adapter_clip.py:117-119 (Q13)."""
    return "adaptmlp" in name or "lora" in name


# ----------------------------------------------------------------------------- primitives
def layer_norm(x, w, b, eps=1e-5):
    """model.py:194-200 — LayerNorm evaluated in fp32."""
    return F.layer_norm(x.float(), (x.shape[-1],), w, b, eps)


def quick_gelu(x):
    """model.py:203-206."""
    return x * torch.sigmoid(1.702 * x)


def linear(x, w, b=None, rt=identity, fp8=False):
    """F.linear with operands rounded at the GEMM input (fp32 accumulate). fp8=True marks the
    frozen-backbone GEMMs (QKV, c_fc, c_proj) that an fp8 rounding hook (``fp8_rounding``)
    evaluates as block-scaled e4m3 GEMMs, forward and input-gradient (``Fp8Linear``)."""
    if fp8 and getattr(rt, "fp8", False):
        y = Fp8Linear.apply(x, w)
    else:
        y = rt(x) @ rt(w).t()
    return y if b is None else y + b


# ----------------------------------------------------------------------------- fp8 rounding
# The block-scaled fp8 operand format of the MI355X fp8 GEMMs (BASELINE config 5 runs MaPLe's
# frozen backbone in fp8; the reference's own MaPLe casts it to fp16, models/maple_clip/
# model.py:749-772, 826). Restated from the OCP Microscaling (MX) v1.0 definition: blocks of 32
# consecutive elements along the reduction axis share an E8M0 scale X = 2^(floor(log2 amax) -
# emax_elem) with emax_elem = 8 for e4m3 (largest normal 448 = 1.75 * 2^8); each element is
# RNE(x / X) in OCP e4m3fn, saturated to +-448 (the conversion torch.float8_e4m3fn implements).
# Build choices beyond the spec, mirrored by the kernels: the scale exponent is clamped to
# [-126, 126]; a block whose amax is 0 or below the f32 normal range gets scale byte 0 and
# zero values.
def fp8_scale_bytes(amax):
    """E8M0 byte of each block's scale from its amax (f32 tensor)."""
    e = (amax.float().contiguous().view(torch.int32) >> 23) & 0xFF
    b = (e - 8).clamp(1, 253)
    return torch.where(e == 0, torch.zeros_like(b), b)


def quant_fp8(x):
    """x [..., K] (K % 32 == 0) -> (codes uint8 [..., K], scale bytes uint8 [..., K/32],
    dequantised f32 [..., K])."""
    *lead, K = x.shape
    xb = x.detach().float().reshape(*lead, K // 32, 32)
    byte = fp8_scale_bytes(xb.abs().amax(-1))
    inv = torch.where(byte == 0, torch.zeros_like(byte, dtype=torch.float32),
                      torch.exp2((127 - byte).float()))
    q = (xb * inv[..., None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    deq = q.float() * torch.exp2((byte - 127).float())[..., None]
    deq = torch.where(byte[..., None] == 0, torch.zeros_like(deq), deq)
    return (q.view(torch.uint8).reshape(*lead, K), byte.to(torch.uint8),
            deq.reshape(*lead, K))


def fp8_round(x):
    """Value of x after the fp8 round trip along its last axis (no gradient path)."""
    return quant_fp8(x)[2]


class Fp8Linear(torch.autograd.Function):
    """y = fp8(x) @ fp8(W)^T with both operands quantised along K (the forward fp8 GEMM);
    dx = fp8(dy) @ fp8(W^T)^T with dy and W^T quantised along N (the input-gradient fp8 GEMM, W
    transposed and quantised once per checkpoint). W is frozen: no weight gradient."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(w)
        return fp8_round(x) @ fp8_round(w).t()

    @staticmethod
    def backward(ctx, dy):
        (w,) = ctx.saved_tensors
        return fp8_round(dy) @ fp8_round(w.t().contiguous()).t(), None


def fp8_rounding(base=None):
    """A rounding hook for the oracle's ``rt`` argument: ``base`` (default round_bf16) everywhere,
    plus block-scaled fp8 GEMMs where ``linear(..., fp8=True)``."""
    base = round_bf16 if base is None else base

    def rt(x):
        return base(x)
    rt.fp8 = True
    if hasattr(base, "resid"):
        rt.resid = base.resid
    return rt


def prompt_tower_resid(cfg: ClipConfig, rt):
    """The frozen prompt towers' residual rounding (MVP, MaPLe): IEEE half on the MI355X image
    tower at widths 512 / 768 (lcclip ImageTower._resid16), forward only (straight-through: the
    residual gradient stays f32 there); identity for the fp32 oracle. The reference casts the
    prompt rows to the stream's dtype (mvp_clip.py:256-257, maple.py:243), so they are rounded
    with the stream."""
    return round_f16 if cfg.vision_width in (512, 768) and hasattr(rt, "resid") else identity


def merged_lora_weight(w, a, bmat, scaling, rt=identity):
    """W + scaling * B @ A, rounded once: the MI355X path merges the rank-r update into the
    frozen weight before the GEMM. Algebraically identical to lora.py:837-839 / 1072-1074
    (F.linear(x, W) + F.linear(F.linear(x, A), B) * scaling)."""
    return rt(w + scaling * (bmat @ a))


def attention_core(q, k, v, scale, causal, rt=identity):
    """lora.py:950 (q * scaling), 1043 (bmm), 1047-1051 (additive -inf mask), 1063 (softmax),
    1068 (bmm). q,k,v: [N, H, L, dh]. With rt=round_bf16 it mirrors the HIP kernel: S in fp32
    from bf16 q,k; P = exp(S - max) rounded to bf16 for the PV product; the row sum l is taken
    from the unrounded fp32 exponentials; O = (P_bf16 @ V) / l, rounded to bf16."""
    q, k, v = rt(q), rt(k), rt(v)
    if getattr(rt, "attn", None) is not None:
        return rt.attn(q, k, v, scale, causal)
    s = (q @ k.transpose(-1, -2)) * scale
    if causal:
        L = s.shape[-1]
        mask = torch.full((L, L), float("-inf")).triu_(1)  # model.py:926-932
        s = s + mask
    m = s.amax(dim=-1, keepdim=True)
    p = torch.exp(s - m)
    l = p.sum(dim=-1, keepdim=True)
    o = (rt(p) @ v) / l
    return rt(o)


def mha(x, p, pre, n_head, causal, lora_scaling=None, rt=identity):
    """Self-attention for x [N, L, D] (batch-first internally; the reference's sequence-first
    layout, model.py:767, is not observable). LoRA variant when the *_lora_* params exist:
    qkv = F.linear(x, W, b) + F.linear(F.linear(x, A), B) * scaling (lora.py:837-839),
    out = F.linear(o, Wo, bo) + F.linear(F.linear(o, Ao), Bo) * scaling (lora.py:1072-1074).
    Returns the attention output BEFORE any rounding of the out-projection result."""
    N, L, D = x.shape
    dh = D // n_head
    w_in = p[pre + "attn.in_proj_weight"]
    w_out = p[pre + "attn.out_proj.weight"]
    lora = (pre + "attn.in_proj_weight_lora_A") in p
    if lora:
        w_in = merged_lora_weight(w_in, p[pre + "attn.in_proj_weight_lora_A"],
                                  p[pre + "attn.in_proj_weight_lora_B"], lora_scaling, rt)
        w_out = merged_lora_weight(w_out, p[pre + "attn.out_proj.lora_A"],
                                   p[pre + "attn.out_proj.lora_B"], lora_scaling, rt)
    qkv = rt(linear(x, w_in, p[pre + "attn.in_proj_bias"], rt, fp8=True))
    q, k, v = qkv.chunk(3, dim=-1)                                   # lora.py:840

    def heads(t):                                                     # lora.py:1002-1006
        return t.reshape(N, L, n_head, dh).permute(0, 2, 1, 3)
    o = attention_core(heads(q), heads(k), heads(v), dh ** -0.5, causal, rt)
    o = o.permute(0, 2, 1, 3).reshape(N, L, D)                        # lora.py:1070-1071
    return linear(o, w_out, p[pre + "attn.out_proj.bias"], rt)


def adapter(z, p, pre, scale=0.1, dropout_mask=None, rt=identity):
    """adapter.py:53-72 with adapter_layernorm_option='none' (model.py:436):
    out = z + scale * up(dropout(relu(down(z)))). ``dropout_mask`` (already divided by keep
    probability) replaces F.dropout when given; None means eval / p = 0."""
    gq = getattr(rt, "bwd", identity)  # dpre stored as bf16 (peft.hip adapter backward)
    d = torch.relu(gq(linear(z, p[pre + "adaptmlp.down_proj.weight"],
                             p[pre + "adaptmlp.down_proj.bias"], rt)))
    if dropout_mask is not None:
        d = d * dropout_mask
    u = linear(d, p[pre + "adaptmlp.up_proj.weight"], p[pre + "adaptmlp.up_proj.bias"], rt)
    return z + scale * u


def block(x, p, pre, n_head, causal, variant, lora_scaling=0.25, rt=identity, masks=None,
          xr=identity):
    """ResidualAttentionBlock{,_LoRA} forward (model.py:233-236) and _Adapter forward
    (model.py:439-442; one adapter module reused for both sub-blocks, Q6). x is the residual
    stream [N, L, D]; xr rounds it after each residual add (the half residual stream)."""
    # gq: the backward's bf16 gradient stores (rt.bwd; identity for the fp32 oracle and the
    # straight-through round_bf16): each sub-block reads the bf16 copy of the residual stream's
    # gradient (dx_midb / the layer's output pair, engine.py BlockStack.backward; the gradient
    # itself is f32 or, through xr, half);
    # dz, dO, da (c_proj dX x QuickGELU'), dh (c_fc dX, QKV dX) are bf16
    gq = getattr(rt, "bwd", identity)
    gelu = getattr(rt, "gelu", quick_gelu)
    h = gq(rt(layer_norm(x, p[pre + "ln_1.weight"], p[pre + "ln_1.bias"])))
    a = mha(h, p, pre, n_head, causal, lora_scaling if variant == "lora" else None, rt)
    if variant == "adapter":
        m0 = None if masks is None else masks[0]
        x = xr(x + gq(adapter(gq(rt(a)), p, pre, dropout_mask=m0, rt=rt)))
    else:
        x = xr(x + gq(a))
    h2 = gq(rt(layer_norm(x, p[pre + "ln_2.weight"], p[pre + "ln_2.bias"])))
    f = rt(gelu(gq(linear(h2, p[pre + "mlp.c_fc.weight"], p[pre + "mlp.c_fc.bias"], rt,
                          fp8=True))))
    m = linear(f, p[pre + "mlp.c_proj.weight"], p[pre + "mlp.c_proj.bias"], rt, fp8=True)
    if variant == "adapter":
        m1 = None if masks is None else masks[1]
        x = xr(x + gq(adapter(gq(rt(m)), p, pre, dropout_mask=m1, rt=rt)))
    else:
        x = xr(x + gq(m))
    return x


def tower_variant(method: str, peft_encoder: str, modal: str) -> str:
    if peft_on(peft_encoder, modal) and method in ("lora", "adapter"):
        return method
    return "vanilla"


def encode_image(img, p, cfg: ClipConfig, method="vanilla", peft_encoder="none", rt=identity,
                 masks=None):
    """VisualTransformer.forward, model.py:755-787 (Q1: blocks called as blk(x))."""
    N = img.shape[0]
    W, P = cfg.vision_width, cfg.vision_patch_size
    g = cfg.grid
    # conv1 (k = s = P, no bias) == GEMM over [3*P*P] patches in (c, kh, kw) order
    patches = img.reshape(N, 3, g, P, g, P).permute(0, 2, 4, 1, 3, 5).reshape(N, g * g, 3 * P * P)
    x = linear(patches, p["visual.conv1.weight"].reshape(W, -1), None, rt)      # :756-758
    cls = p["visual.class_embedding"].reshape(1, 1, W).expand(N, 1, W)
    x = torch.cat([cls, x], dim=1)                                              # :759-763
    x = x + p["visual.positional_embedding"]                                    # :764
    variant = tower_variant(method, peft_encoder, "image")
    # the MI355X image tower's half residual stream (round_bf16.resid above): the adapter and
    # LoRA towers (their gradient in half too, in the backward-faithful rounding), the frozen
    # tower (forward)
    xr = identity
    if cfg.vision_width in (512, 768) and hasattr(rt, "resid"):
        xr = rt.resid if variant in ("adapter", "lora") else round_f16
    x = xr(layer_norm(x, p["visual.ln_pre.weight"], p["visual.ln_pre.bias"]))  # :766
    vis, _ = tower_prefixes(cfg)
    for i, pre in enumerate(vis):
        x = block(x, p, pre, cfg.vision_heads, False, variant, rt=rt,
                  masks=None if masks is None else masks[i], xr=xr)
    tail = getattr(rt, "tail", rt)  # rounding of ln_post's output and the projection GEMM
    x = tail(layer_norm(x[:, 0, :], p["visual.ln_post.weight"], p["visual.ln_post.bias"]))  # :783
    # the feature gradient is cast to 16 bits before the projection's backward GEMM
    return getattr(rt, "top", identity)(
        getattr(rt, "bwd", identity)(linear(x, p["visual.proj"].t(), None, tail)))  # :785


def encode_text(tokens, p, cfg: ClipConfig, method="vanilla", peft_encoder="none", rt=identity,
                masks=None):
    """CLIP.encode_text, model.py:941-956; causal mask model.py:926-932; EOT pooling by
    argmax of the token ids (Q11). ln_final is row-local, so gathering the EOT row first and
    normalising it equals normalising all rows then gathering."""
    C = tokens.shape[0]
    x = p["token_embedding.weight"][tokens] + p["positional_embedding"]
    variant = tower_variant(method, peft_encoder, "text")
    _, txt = tower_prefixes(cfg)
    for i, pre in enumerate(txt):
        x = block(x, p, pre, cfg.transformer_heads, True, variant, rt=rt,
                  masks=None if masks is None else masks[i])
    eot = tokens.argmax(dim=-1)
    x = x[torch.arange(C), eot]
    tail = getattr(rt, "tail", rt)  # rounding of ln_final's output and the projection GEMM
    x = tail(layer_norm(x, p["ln_final.weight"], p["ln_final.bias"]))
    return getattr(rt, "top", identity)(
        getattr(rt, "bwd", identity)(linear(x, p["text_projection"].t(), None, tail)))


def clip_logits(img_f, txt_f, logit_scale):
    """model.py:966-974: L2-normalise, logits = exp(logit_scale) * I @ T^T."""
    i = img_f / img_f.norm(dim=-1, keepdim=True)
    t = txt_f / txt_f.norm(dim=-1, keepdim=True)
    return logit_scale.exp() * i @ t.t(), i, t


def adapter_clip_forward(img, tokens, p, cfg, method, peft_encoder, rt=identity,
                         img_masks=None, txt_masks=None, rt_text=None):
    """AdapterCLIP.forward, models/adapter_clip.py:94-100 -> (probs, img_f, txt_f). rt_text:
    the text tower's rounding hook when it differs from the image tower's (default rt)."""
    fi = encode_image(img, p, cfg, method, peft_encoder, rt, img_masks)
    ft = encode_text(tokens, p, cfg, method, peft_encoder, rt if rt_text is None else rt_text,
                     txt_masks)
    logits, i, t = clip_logits(fi, ft, p["logit_scale"])
    return logits.softmax(dim=-1), i, t


def loss_on_probs(probs, y):
    """nn.CrossEntropyLoss()(probs, y) — applied to probabilities (Q5)."""
    return F.cross_entropy(probs, y)


def adamw_step(params, grads, state, lr=5e-4, betas=(0.9, 0.999), eps=1e-8, wd=1e-5):
    """One torch.optim.AdamW step (utils/train_utils.py:27-28), written out so the semantics
    are explicit. state: dict name -> (step, m, v)."""
    b1, b2 = betas
    out = {}
    for n, prm in params.items():
        g = grads[n]
        step, m, v = state.get(n, (0, torch.zeros_like(prm), torch.zeros_like(prm)))
        step += 1
        prm = prm * (1 - lr * wd)
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = (v / bc2).sqrt() + eps
        prm = prm - (lr / bc1) * m / denom
        state[n] = (step, m, v)
        out[n] = prm
    return out


def train_step(img, tokens, y, p, cfg, method, peft_encoder, rt=identity, lr=5e-4, state=None,
               rt_text=None):
    """methods/adapter_clip.py:86-96 at p=0 dropout: fwd -> CE(probs) -> bwd -> AdamW.
    state: the AdamW state carried across steps (None: a fresh optimizer).
    Returns (loss, probs, img_f, txt_f, grads, new_params)."""
    leaves = {n: t.detach().clone().requires_grad_(is_trainable(n)) for n, t in p.items()}
    probs, fi, ft = adapter_clip_forward(img, tokens, leaves, cfg, method, peft_encoder, rt,
                                         rt_text=rt_text)
    loss = loss_on_probs(probs, y)
    train = {n: t for n, t in leaves.items() if t.requires_grad}
    if not train:  # vanilla blocks: nothing is trainable (the freeze filter leaves no params)
        return loss.detach(), probs.detach(), fi.detach(), ft.detach(), {}, {}
    grads = dict(zip(train.keys(), torch.autograd.grad(loss, list(train.values()))))
    new = adamw_step({n: t.detach() for n, t in train.items()}, grads,
                     {} if state is None else state, lr=lr)
    return loss.detach(), probs.detach(), fi.detach(), ft.detach(), grads, new


def online_loop(task_batches, images, labels, class_tokens, p, cfg, method="adapter",
                peft_encoder="both", online_iter=3, lr=5e-4, rt=identity, rt_text=None):
    """The online loop of methods/_trainer.py:320-357 + methods/adapter_clip.py:34-107, restated
    for the trajectory parity test (replay memory off, visible_classes='batch', p = 0 dropout,
    inputs already transformed). task_batches: per task, the list of sample-index lists the
    sampler yields; class_tokens: [n_classes, L] token ids in class-id order.
      online_before_task: a fresh AdamW per task (adapter_clip.py:115-127, Q14)
      online_step: exposed classes += new labels (_trainer.py:404-413), the batch's class list
                   = its distinct labels in first-seen order (adapter_clip.py:263-283), then
                   online_iter x online_train on clones of the batch (:42-46)
      online_train: y -> index in the batch class list (:75-76), tokens of that list (:84),
                   fwd + CE-on-probs + bwd + AdamW (:86-96)
    Returns [(loss, {trainable name: tensor after the step})] per optimizer step."""
    params = {n: t.detach().clone() for n, t in p.items()}
    exposed, out = [], []
    for batches in task_batches:
        state = {}
        for b in batches:
            ys = [int(v) for v in labels[b].tolist()]
            for y in ys:
                if y not in exposed:
                    exposed.append(y)
            batch_list = []
            for y in ys:
                if y not in batch_list:
                    batch_list.append(y)
            for _ in range(online_iter):
                yi = torch.tensor([batch_list.index(y) for y in ys], dtype=torch.long)
                tok = class_tokens[torch.tensor(batch_list)]
                loss, _, _, _, _, new = train_step(images[b], tok, yi, params, cfg, method,
                                                   peft_encoder, rt, lr, state, rt_text=rt_text)
                params.update(new)
                out.append((loss, {n: t.clone() for n, t in new.items()}))
    return out


# ----------------------------------------------------------------------------- train transform
def train_transform(x, inp_size, padding, crop_i, crop_j, flip, mean, std, quantize=True,
                    aug_ops=()):
    """methods/_trainer.py:212-242 on a batch tensor (torchvision tensor semantics: one parameter
    draw per call, shared by the batch): the autoaug branch's uint8 round trip (:216, :229) with
    the drawn AutoAugment ops between (aug_ops, see ``autoaugment``), Resize((S, S)) —
    torchvision's F.resize is F.interpolate(bilinear, align_corners=False) (antialias is inert
    when upsampling) —, RandomCrop(S, padding) = zero F.pad then the [i:i+S, j:j+S] window,
    hflip, Normalize ((x - mean) / std)."""
    if aug_ops:
        x = autoaugment(x, aug_ops)
    elif quantize:
        x = (x * 255).to(torch.uint8).to(torch.float32) / 255
    x = F.interpolate(x, size=(inp_size, inp_size), mode="bilinear", align_corners=False)
    x = F.pad(x, (padding, padding, padding, padding), value=0.0)
    x = x[:, :, crop_i:crop_i + inp_size, crop_j:crop_j + inp_size]
    if flip:
        x = x.flip(-1)
    m = torch.tensor(mean, dtype=x.dtype).view(1, -1, 1, 1)
    s = torch.tensor(std, dtype=x.dtype).view(1, -1, 1, 1)
    return (x - m) / s


# AutoAugment ops (torchvision 0.16.2 transforms/autoaugment.py _apply_op over
# transforms/_functional_tensor.py, restated; torchvision is not installed here, so parity with
# torchvision itself is unpinned). Images are uint8-valued int64 tensors [n, C, H, W]; every f32
# expression is evaluated op by op in torch's order so the MI355X kernel (transform.hip
# autoaug_kernel) can match bit for bit. Where torchvision evaluates with a bmm / conv2d whose
# summation order is library-defined (the affine grid, the sharpness blur), the order fixed
# here is left-to-right.
def _f32(v):
    return torch.tensor(v, dtype=torch.float32)


def _aa_blend(img, other, ratio):
    """_blend: (ratio * img + (1 - ratio) * other).clamp(0, 255).to(uint8)."""
    r1, r2 = _f32(ratio), _f32(1.0 - ratio)
    return (r1 * img.float() + r2 * other).clamp(0, 255).to(torch.uint8).long()


def _aa_gray(img):
    """rgb_to_grayscale on uint8: (0.2989 r + 0.587 g + 0.114 b).to(uint8)."""
    r, g, b = img[:, 0].float(), img[:, 1].float(), img[:, 2].float()
    return (_f32(0.2989) * r + _f32(0.587) * g + _f32(0.114) * b).to(torch.uint8).long()


def _aa_affine_matrix(center, angle, translate, scale, shear):
    """_get_inverse_affine_matrix (doubles)."""
    rot, sx, sy = math.radians(angle), math.radians(shear[0]), math.radians(shear[1])
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    m = [v / scale for v in (d, -b, 0.0, -c, a, 0.0)]
    m[2] += m[0] * (-cx - tx) + m[1] * (-cy - ty) + cx
    m[5] += m[3] * (-cx - tx) + m[4] * (-cy - ty) + cy
    return m


def _aa_affine(img, m):
    """F_t.affine / F_t.rotate with NEAREST and no fill: _gen_affine_grid + grid_sample
    (align_corners=False, zeros padding) + round to uint8."""
    n, C, H, W = img.shape
    t = torch.tensor(m, dtype=torch.float32)
    hw, hh = _f32(0.5 * W), _f32(0.5 * H)
    r = [t[0] / hw, t[1] / hw, t[2] / hw, t[3] / hh, t[4] / hh, t[5] / hh]
    xs = torch.linspace(-W * 0.5 + 0.5, W * 0.5 + 0.5 - 1, W).view(1, W).expand(H, W)
    ys = torch.linspace(-H * 0.5 + 0.5, H * 0.5 + 0.5 - 1, H).view(H, 1).expand(H, W)
    gx = (xs * r[0] + ys * r[1]) + r[2]
    gy = (xs * r[3] + ys * r[4]) + r[5]
    ix = torch.round(((gx + 1) * W - 1) / 2).long()   # grid_sampler_unnormalize + nearbyint
    iy = torch.round(((gy + 1) * H - 1) / 2).long()
    ok = (ix >= 0) & (ix < W) & (iy >= 0) & (iy < H)
    flat = (iy.clamp(0, H - 1) * W + ix.clamp(0, W - 1)).view(-1)
    out = img.reshape(n, C, H * W)[:, :, flat].reshape(n, C, H, W)
    return torch.where(ok, out, torch.zeros_like(out))


def _aa_equalize_channel(ch):
    hist = torch.bincount(ch.reshape(-1), minlength=256)
    nz = hist[hist != 0]
    step = int(nz[:-1].sum()) // 255
    if step == 0:
        return ch
    lut = (torch.cumsum(hist, 0) + step // 2) // step
    lut = torch.nn.functional.pad(lut, [1, 0])[:-1].clamp(0, 255)
    return lut[ch]


def aa_apply_op(img, op, mag):
    """_apply_op(img, op_name, magnitude) for NEAREST interpolation and fill=None."""
    n, C, H, W = img.shape
    if op == "ShearX":
        return _aa_affine(img, _aa_affine_matrix([-0.5 * W, -0.5 * H], 0.0, [0.0, 0.0], 1.0,
                                                 [math.degrees(math.atan(mag)), 0.0]))
    if op == "ShearY":
        return _aa_affine(img, _aa_affine_matrix([-0.5 * W, -0.5 * H], 0.0, [0.0, 0.0], 1.0,
                                                 [0.0, math.degrees(math.atan(mag))]))
    if op == "TranslateX":
        return _aa_affine(img, _aa_affine_matrix([0.0, 0.0], 0.0, [float(int(mag)), 0.0], 1.0,
                                                 [0.0, 0.0]))
    if op == "TranslateY":
        return _aa_affine(img, _aa_affine_matrix([0.0, 0.0], 0.0, [0.0, float(int(mag))], 1.0,
                                                 [0.0, 0.0]))
    if op == "Rotate":
        return _aa_affine(img, _aa_affine_matrix([0.0, 0.0], -mag, [0.0, 0.0], 1.0, [0.0, 0.0]))
    if op == "Brightness":
        return _aa_blend(img, torch.zeros(()), 1.0 + mag)
    if op == "Color":
        return _aa_blend(img, _aa_gray(img).float().unsqueeze(1), 1.0 + mag)
    if op == "Contrast":
        mean = _aa_gray(img).float().mean(dim=(-2, -1), keepdim=True).unsqueeze(1)
        return _aa_blend(img, mean, 1.0 + mag)
    if op == "Sharpness":
        if H <= 2 or W <= 2:
            return img
        k = torch.ones(3, 3)
        k[1, 1] = 5.0
        k = k / k.sum()
        f = img.float()
        s = torch.zeros(n, C, H - 2, W - 2)
        for di in range(3):
            for dj in range(3):
                s = s + f[:, :, di:di + H - 2, dj:dj + W - 2] * k[di, dj]
        blur = img.clone()
        blur[:, :, 1:-1, 1:-1] = torch.round(s).long()
        return _aa_blend(img, blur.float(), 1.0 + mag)
    if op == "Posterize":
        return img & ((-int(2 ** (8 - int(mag)))) & 0xFF)
    if op == "Solarize":
        return torch.where(img.float() >= _f32(mag), 255 - img, img)
    if op == "AutoContrast":
        mn = img.amin(dim=(-2, -1), keepdim=True).float()
        mx = img.amax(dim=(-2, -1), keepdim=True).float()
        scale = 255 / (mx - mn)
        bad = ~torch.isfinite(scale)
        mn = torch.where(bad, torch.zeros_like(mn), mn)
        scale = torch.where(bad, torch.ones_like(scale), scale)
        return ((img.float() - mn) * scale).clamp(0, 255).to(torch.uint8).long()
    if op == "Equalize":
        return torch.stack([torch.stack([_aa_equalize_channel(img[i, c]) for c in range(C)])
                            for i in range(n)])
    if op == "Invert":
        return 255 - img
    raise ValueError(op)


def autoaugment(x, ops):
    """x f32 [n, C, H, W] in [0, 1] -> (x*255).type(uint8) -> the active ops in order ->
    .float() / 255 (methods/_trainer.py:216-229)."""
    img = (x * 255).to(torch.uint8).long()
    for op, mag in ops:
        img = aa_apply_op(img, op, mag)
    return img.to(torch.float32) / 255


def patchify(img, patch):
    """conv1's im2col (model.py:756): [n, C, S, S] -> [n*(S/P)^2, C*P*P] in (c, ky, kx) order."""
    n, C, S, _ = img.shape
    g = S // patch
    t = img.reshape(n, C, g, patch, g, patch).permute(0, 2, 4, 1, 3, 5)
    return t.reshape(n * g * g, C * patch * patch)


# ----------------------------------------------------------------------------- synthetic data
def synthetic_images(n, res=224, seed=0):
    """U[0,1) images normalised with the CIFAR-100 statistics
    (datasets/__init__.py:38-39)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, 3, res, res, generator=g)
    mean = torch.tensor([0.5071, 0.4867, 0.4408]).view(1, 3, 1, 1)
    std = torch.tensor([0.2675, 0.2565, 0.2761]).view(1, 3, 1, 1)
    return (x - mean) / std


def synthetic_tokens(c, context_length=77, seed=0, vocab=49408):
    """C rows [SOT, t_1..t_k, EOT, 0...], k ~ U{6..12}, t ~ U{256..49405}.
    SOT/EOT are the two highest ids (49406/49407 for the CLIP vocab), so EOT pooling by argmax
    (model.py:953-954) finds the EOT position."""
    g = torch.Generator().manual_seed(seed + 7)
    sot, eot = vocab - 2, vocab - 1
    lo = min(256, vocab // 4)
    out = torch.zeros(c, context_length, dtype=torch.long)
    for i in range(c):
        k = int(torch.randint(6, 13, (1,), generator=g))
        body = torch.randint(lo, sot, (k,), generator=g)
        out[i, 0] = sot
        out[i, 1:1 + k] = body
        out[i, 1 + k] = eot
    return out


def synthetic_state_dict(cfg: ClipConfig, method="vanilla", peft_encoder="none", seed=1234,
                         peft_nonzero=True):
    """Seeded weights in the reference's state-dict layout with CLIP-like statistics
    (model.py:852-885; Linear-style fan-in scaling elsewhere). With peft_nonzero the LoRA B and
    adapter up weights are NONZERO so the PEFT forward and dW paths are exercised (SURVEY.md
    §8(c): zero inits would hide bugs); biases are nonzero too."""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for name, shape in param_shapes(cfg, method, peft_encoder).items():
        if name == "logit_scale":
            sd[name] = torch.tensor(math.log(1 / 0.07))
            continue
        if name.endswith("ln_1.weight") or name.endswith("ln_2.weight") or name.endswith(
                ("ln_pre.weight", "ln_post.weight", "ln_final.weight")):
            sd[name] = 1.0 + 0.1 * torch.randn(shape, generator=g)
            continue
        if name.endswith("bias") and "ln_" in name:
            sd[name] = 0.05 * torch.randn(shape, generator=g)
            continue
        if name.endswith("bias"):
            sd[name] = 0.02 * torch.randn(shape, generator=g)
            continue
        if "lora_B" in name or "up_proj.weight" in name:
            std = 0.05 if peft_nonzero else 0.0
            sd[name] = std * torch.randn(shape, generator=g)
            continue
        if name in ("token_embedding.weight",):
            sd[name] = 0.02 * torch.randn(shape, generator=g)
            continue
        if name == "positional_embedding":
            sd[name] = 0.01 * torch.randn(shape, generator=g)
            continue
        if len(shape) == 1:
            sd[name] = (shape[0] ** -0.5) * torch.randn(shape, generator=g)
            continue
        fan_in = 1
        for s in shape[1:]:
            fan_in *= s
        if name in ("visual.proj", "text_projection", "visual.positional_embedding"):
            fan_in = shape[0]
        sd[name] = (fan_in ** -0.5) * torch.randn(shape, generator=g)
    return sd


TINY = ClipConfig(embed_dim=64, image_resolution=64, vision_layers=2, vision_width=128,
                  vision_patch_size=16, context_length=77, vocab_size=512, transformer_width=64,
                  transformer_heads=1, transformer_layers=2)


# ------------------------------------------------------------------------------------------------
# MVP-CLIP (models/mvp_clip.py, BASELINE config 3): frozen vanilla backbone, prompt tuning.
def mvp_embed(img, p, cfg: ClipConfig, rt=identity):
    """conv1 + CLS/pos + ln_pre, batch-first [N, L, W] (mvp_clip.py:197-210 = model.py:756-766)."""
    N = img.shape[0]
    W, P = cfg.vision_width, cfg.vision_patch_size
    g = cfg.grid
    patches = img.reshape(N, 3, g, P, g, P).permute(0, 2, 4, 1, 3, 5).reshape(N, g * g, 3 * P * P)
    x = linear(patches, p["visual.conv1.weight"].reshape(W, -1), None, rt)
    cls = p["visual.class_embedding"].reshape(1, 1, W).expand(N, 1, W)
    x = torch.cat([cls, x], dim=1) + p["visual.positional_embedding"]
    return layer_norm(x, p["visual.ln_pre.weight"], p["visual.ln_pre.bias"])


def mvp_prompt_layers(g_prompt, e_prompt, pos_g, len_g, pos_e, len_e, n_layers):
    """{layer: [B, P, W]} appended at that layer: g then e (mvp_clip.py:158-172; the prompt
    tensors are viewed as [B, -1, len, W] and indexed by the layer's position in pos_*)."""
    B, _, W = g_prompt.shape
    g = g_prompt.reshape(B, -1, len_g, W)
    e = e_prompt.reshape(B, -1, len_e, W)
    out = {}
    for n in range(n_layers):
        parts = []
        if n in pos_g:
            parts.append(g[:, list(pos_g).index(n)])
        if n in pos_e:
            parts.append(e[:, list(pos_e).index(n)])
        if parts:
            out[n] = torch.cat(parts, dim=1)
    return out


def mvp_forward(img, tokens, p, cfg: ClipConfig, mvp: dict, pos_g=(0, 1), len_g=5,
                pos_e=(2, 3, 4), len_e=20, use_last_layer=True, use_mask=True, rt=identity,
                rt_text=None):
    """CLIP_MVP.forward (mvp_clip.py:282-288) over forward_features (:182-264) and forward_head
    (:266-280), prompt_func 'prompt_tuning', selection_size 1, use_contrastiv False.
    mvp: {'key' [pool, W], 'mask' [pool, n_classes], 'g_prompts' [1, G, W], 'e_prompts'
    [pool, E, W]}. Returns (logits [B, C] (masked when use_mask), similarity_loss, image
    features [B, E], text features [C, E], mask [B, C], topk [B, 1]). rt_text: the text
    tower's rounding when it differs from the image tower's (the IEEE-half text tower)."""
    vis, _ = tower_prefixes(cfg)
    xr = prompt_tower_resid(cfg, rt)
    x0 = xr(mvp_embed(img, p, cfg, rt))
    B, N, W = x0.shape
    with torch.no_grad():                                                       # :196-218
        q = x0.clone()
        stop = len(vis) if use_last_layer else len(vis) - 1
        for pre in vis[:stop]:
            q = block(q, p, pre, cfg.vision_heads, False, "vanilla", rt=rt, xr=xr)
        query = layer_norm(q[:, 0, :], p["visual.ln_post.weight"], p["visual.ln_post.bias"])
    distance = 1 - F.cosine_similarity(query.unsqueeze(1), mvp["key"], dim=-1)  # :224-225
    topk = distance.topk(1, dim=1, largest=False)[1]                            # :231-232
    distance = distance[torch.arange(B).unsqueeze(1), topk].squeeze(1)          # :233-235
    e_prompts = mvp["e_prompts"][topk].squeeze(1)                               # :236
    mask = mvp["mask"][topk].mean(1)                                            # :237
    sim_loss = distance.mean()                                                  # :248
    g_prompts = mvp["g_prompts"][0].repeat(B, 1, 1)                             # :250
    prompts = mvp_prompt_layers(g_prompts, e_prompts, pos_g, len_g, pos_e, len_e, len(vis))
    x = x0
    for i, pre in enumerate(vis):                                               # :163-175
        if i in prompts:
            x = torch.cat([x, xr(prompts[i])], dim=1)
        x = block(x, p, pre, cfg.vision_heads, False, "vanilla", rt=rt, xr=xr)
        x = x[:, :N]
    x = rt(layer_norm(x[:, 0, :], p["visual.ln_post.weight"], p["visual.ln_post.bias"]))
    img_f = linear(x, p["visual.proj"].t(), None, rt)                          # :259-261
    txt_f = encode_text(tokens, p, cfg, "vanilla", "none",
                        rt if rt_text is None else rt_text)                     # :192
    C = tokens.shape[0]
    mask = torch.sigmoid(mask) * 2.0                                           # :263
    logits, _, _ = clip_logits(img_f, txt_f, p["logit_scale"])                 # :266-280
    if use_mask:
        logits = logits * mask[:, :C]                                          # :286-287
    return logits, sim_loss, img_f, txt_f, mask[:, :C], topk


def mvp_params(cfg: ClipConfig, pool=10, n_classes=100, len_g=5, n_g=2, len_e=20, n_e=3, seed=7):
    """MVP trainable tensors with the reference's shapes (mvp_clip.py:84-94): key randn,
    mask zeros - 1 (here randomised around -1 so the mask gradient path is exercised),
    g_prompts [1, n_g*len_g, W], e_prompts [pool, n_e*len_e, W] randn."""
    g = torch.Generator().manual_seed(seed)
    W = cfg.vision_width
    return {
        "key": torch.randn(pool, W, generator=g),
        "mask": -1.0 + 0.5 * torch.randn(pool, n_classes, generator=g),
        "g_prompts": torch.randn(1, n_g * len_g, W, generator=g),
        "e_prompts": torch.randn(pool, n_e * len_e, W, generator=g),
    }


TINY_MVP = ClipConfig(embed_dim=64, image_resolution=64, vision_layers=6, vision_width=128,
                      vision_patch_size=16, context_length=77, vocab_size=512, transformer_width=64,
                      transformer_heads=1, transformer_layers=2)


# ------------------------------------------------------------------------------------------------
# MaPLe (models/maple.py + models/maple_clip/model.py, BASELINE config 5): frozen backbone,
# multi-modal prompts. mp: {'ctx' [n_ctx, Dt], 'proj.weight' [Dv, Dt], 'proj.bias' [Dv],
# 'text.{i}' [n_ctx, Dt], 'vproj.{i}.weight' [Dv, Dt], 'vproj.{i}.bias' [Dv]} for i < depth-1.
def maple_forward(img, tokens, p, cfg: ClipConfig, mp: dict, n_ctx=3, depth=3, rt=identity,
                  rt_img=None):
    """MaPLe.forward (maple.py:208-251) -> logits [B, C] (no softmax). rt_img: the image tower's
    rounding hook when it differs from the text tower's (fp8 image tower: fp8_rounding())."""
    rt_img = rt if rt_img is None else rt_img
    C = tokens.shape[0]
    emb = p["token_embedding.weight"][tokens]                                  # maple.py:200-203
    prefix, suffix = emb[:, :1], emb[:, 1 + n_ctx:]                            # :205-206
    ctx = mp["ctx"].unsqueeze(0).expand(C, -1, -1)                             # :158-161
    deep_text = [mp[f"text.{i}"] for i in range(depth - 1)]
    deep_vis = [linear(mp[f"text.{i}"], mp[f"vproj.{i}.weight"], mp[f"vproj.{i}.bias"])
                for i in range(depth - 1)]                                      # :164-169
    shared = linear(mp["ctx"], mp["proj.weight"], mp["proj.bias"])              # :171-172
    # text encoder (maple.py:53-68) with deep prompts at rows 1..n_ctx of layers 1..depth-1
    # (maple_clip/model.py:381-395: prefix x[:1], context, suffix x[1 + n_ctx:])
    x = torch.cat([prefix, ctx, suffix], dim=1) + p["positional_embedding"]     # :134-146, :54
    _, txt = tower_prefixes(cfg)
    for i, pre in enumerate(txt):
        if 1 <= i <= len(deep_text):
            x = torch.cat([x[:, :1], deep_text[i - 1].unsqueeze(0).expand(C, -1, -1),
                           x[:, 1 + n_ctx:]], dim=1)
        x = block(x, p, pre, cfg.transformer_heads, True, "vanilla", rt=rt)
    x = x[torch.arange(C), tokens.argmax(dim=-1)]
    x = rt(layer_norm(x, p["ln_final.weight"], p["ln_final.bias"]))
    txt_f = linear(x, p["text_projection"].t(), None, rt)
    # image encoder (maple_clip/model.py:551-590): shared context appended before ln_pre, deep
    # prompts replacing the last n_ctx rows of layers 1..depth-1 (model.py:364-380)
    N = img.shape[0]
    W, P = cfg.vision_width, cfg.vision_patch_size
    g = cfg.grid
    patches = img.reshape(N, 3, g, P, g, P).permute(0, 2, 4, 1, 3, 5).reshape(N, g * g, 3 * P * P)
    xi = linear(patches, p["visual.conv1.weight"].reshape(W, -1), None, rt_img)
    cls = p["visual.class_embedding"].reshape(1, 1, W).expand(N, 1, W)
    xi = torch.cat([cls, xi], dim=1) + p["visual.positional_embedding"]
    xi = torch.cat([xi, shared.unsqueeze(0).expand(N, -1, -1)], dim=1)        # :568-570
    xr = prompt_tower_resid(cfg, rt_img)
    xi = xr(layer_norm(xi, p["visual.ln_pre.weight"], p["visual.ln_pre.bias"]))  # :575
    vis, _ = tower_prefixes(cfg)
    for i, pre in enumerate(vis):
        if 1 <= i <= len(deep_vis):
            xi = torch.cat([xi[:, :-n_ctx], xr(deep_vis[i - 1]).unsqueeze(0).expand(N, -1, -1)],
                           dim=1)
        xi = block(xi, p, pre, cfg.vision_heads, False, "vanilla", rt=rt_img, xr=xr)
    xi = rt_img(layer_norm(xi[:, 0, :], p["visual.ln_post.weight"], p["visual.ln_post.bias"]))
    img_f = linear(xi, p["visual.proj"].t(), None, rt_img)
    logits, _, _ = clip_logits(img_f, txt_f, p["logit_scale"])                # :244-250
    return logits


def maple_params(cfg: ClipConfig, n_ctx=3, depth=3, seed=9):
    """MaPLe prompt-learner tensors with the reference's shapes and init scales
    (maple.py:94-123: ctx / compound text prompts N(0, 0.02); nn.Linear default init)."""
    g = torch.Generator().manual_seed(seed)
    Dt, Dv = cfg.transformer_width, cfg.vision_width
    mp = {"ctx": 0.02 * torch.randn(n_ctx, Dt, generator=g),
          "proj.weight": (Dt ** -0.5) * torch.randn(Dv, Dt, generator=g),
          "proj.bias": 0.02 * torch.randn(Dv, generator=g)}
    for i in range(depth - 1):
        mp[f"text.{i}"] = 0.02 * torch.randn(n_ctx, Dt, generator=g)
        mp[f"vproj.{i}.weight"] = (Dt ** -0.5) * torch.randn(Dv, Dt, generator=g)
        mp[f"vproj.{i}.bias"] = 0.02 * torch.randn(Dv, generator=g)
    return mp


MAPLE_TO_MODULE = {"ctx": "prompt_learner.ctx", "proj.weight": "prompt_learner.proj.weight",
                   "proj.bias": "prompt_learner.proj.bias",
                   "text.0": "prompt_learner.compound_prompts_text.0",
                   "text.1": "prompt_learner.compound_prompts_text.1",
                   "vproj.0.weight": "prompt_learner.compound_prompt_projections.0.weight",
                   "vproj.0.bias": "prompt_learner.compound_prompt_projections.0.bias",
                   "vproj.1.weight": "prompt_learner.compound_prompt_projections.1.weight",
                   "vproj.1.bias": "prompt_learner.compound_prompt_projections.1.bias"}

# fp8 image tower needs widths in multiples of 256 (the fp8 GEMM's N tiles)
TINY_MAPLE8 = ClipConfig(embed_dim=64, image_resolution=64, vision_layers=4, vision_width=256,
                         vision_patch_size=16, context_length=77, vocab_size=512,
                         transformer_width=64, transformer_heads=1, transformer_layers=3)

TINY_MAPLE = ClipConfig(embed_dim=64, image_resolution=64, vision_layers=4, vision_width=128,
                        vision_patch_size=16, context_length=77, vocab_size=512,
                        transformer_width=64, transformer_heads=1, transformer_layers=3)
