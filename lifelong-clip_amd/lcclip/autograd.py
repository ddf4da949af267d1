"""torch.autograd.Function wrappers that connect the fused tower engines to autograd.

Only the PEFT parameters (LoRA A/B, adapter weights/biases) are passed as Function inputs, so
autograd routes their gradients; the frozen backbone is read from the modules directly.
"""
from __future__ import annotations

import torch

from . import ops
from .engine import ScaledGrads
from .ops import F32


def _check_frozen(stack):
    if torch.is_grad_enabled():
        for p in stack.backbone_params():
            if p.requires_grad:
                raise RuntimeError(
                    "lcclip computes PEFT gradients only: freeze the backbone first (the "
                    "reference does in online_before_task, methods/adapter_clip.py:115-119; "
                    "see lcclip.freeze_backbone)")


class _TowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tower, inp, training, save, *params):
        f, c = tower.forward(inp, save=save, training=training)
        ctx.tower = tower
        ctx.saved_ctx = c
        ctx.params = tower.stack.trainable_params()
        return f

    @staticmethod
    def backward(ctx, df):
        if ctx.saved_ctx is None:
            raise RuntimeError("tower forward ran without saving activations")
        grads = {p: torch.zeros(p.shape, dtype=F32, device=p.device) for p in ctx.params}
        ctx.tower.backward(ctx.saved_ctx, df.contiguous().float(), grads)
        ctx.saved_ctx = None
        return (None, None, None, None, *[grads[p] for p in ctx.params])


def tower_apply(tower, transformer, inp, training):
    stack = tower.stack
    _check_frozen(stack)
    params = stack.trainable_params()
    save = torch.is_grad_enabled() and any(p.requires_grad for p in params)
    return _TowerFn.apply(tower, inp, bool(training), save, *params)


class _StackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, stack, x, n_seq, L, training, save, *params):
        y, saved = stack.forward(x, n_seq, L, save=save, training=training)
        ctx.stack, ctx.saved_list, ctx.n_seq, ctx.L = stack, saved, n_seq, L
        ctx.params = stack.trainable_params()
        return y

    @staticmethod
    def backward(ctx, dy):
        grads = {p: torch.zeros(p.shape, dtype=F32, device=p.device) for p in ctx.params}
        sg = None
        if ctx.stack.dt == torch.float16:
            # IEEE-half storage: the incoming gradient (mostly below half's normal range at
            # ViT-B/16) is scaled by a power of two first and every result divided by it again,
            # as the fused towers do (engine.ScaledGrads; the GradScaler's role,
            # methods/adapter_clip.py:93)
            sg = ScaledGrads(ctx.stack, dy)
            dy, g_run = sg.df, sg.grads
        else:
            dy, g_run = dy.contiguous().float().clone(), grads
        dyb = torch.empty(dy.shape, dtype=ctx.stack.dt, device=dy.device)
        ops.cast_bf16(dy, dyb)
        dx, _ = ctx.stack.backward(ctx.saved_list, dy, dyb, g_run, ctx.n_seq, ctx.L)
        ctx.saved_list = None
        if sg is not None:
            sg.add_to(grads)
            dx = sg.unscaled(dx)
        return (None, dx, None, None, None, None, *[grads[p] for p in ctx.params])


def stack_apply(transformer, x2d, n_seq, L):
    stack = transformer.engine
    _check_frozen(stack)
    params = stack.trainable_params()
    save = torch.is_grad_enabled() and (x2d.requires_grad or any(p.requires_grad for p in params))
    return _StackFn.apply(stack, x2d, n_seq, L, bool(transformer.training), save, *params)


class _HeadFn(torch.autograd.Function):
    """model.py:966-974 (+ models/adapter_clip.py:99 softmax when probs=True)."""

    @staticmethod
    def forward(ctx, img_f, txt_f, logit_scale, probs):
        img_f = img_f.contiguous().float()
        txt_f = txt_f.contiguous().float()
        B, E = img_f.shape
        C = txt_f.shape[0]
        dev = img_f.device
        img_n = torch.empty_like(img_f)
        txt_n = torch.empty_like(txt_f)
        ni = torch.empty(B, dtype=F32, device=dev)
        nt = torch.empty(C, dtype=F32, device=dev)
        ops.l2norm_rows(img_f, img_n, ni)
        ops.l2norm_rows(txt_f, txt_n, nt)
        logits = torch.empty(B, C, dtype=F32, device=dev)
        pr = torch.empty(B, C, dtype=F32, device=dev) if probs else None
        ls = logit_scale.detach().reshape(1).float().contiguous()
        ops.head_logits(img_n, txt_n, ls, logits, pr)
        ctx.save_for_backward(img_n, txt_n, ni, nt, ls, pr if probs else logits)
        ctx.probs = probs
        out = pr if probs else logits
        return out, img_n, txt_n

    @staticmethod
    def backward(ctx, d_out, d_img_n, d_txt_n):
        img_n, txt_n, ni, nt, ls, pr = ctx.saved_tensors
        B, C = d_out.shape
        d_out = d_out.contiguous().float()
        if ctx.probs:
            dlog = torch.empty_like(d_out)
            ops.softmax_bwd_rows(pr, d_out, dlog)
        else:
            dlog = d_out
        d_img = torch.empty_like(img_n)
        d_txt = torch.empty_like(txt_n)
        ops.head_feat_grad(dlog, C, 1, txt_n, img_n, ni, ls, d_img,
                           None if d_img_n is None else d_img_n.contiguous().float())
        ops.head_feat_grad(dlog, 1, C, img_n, txt_n, nt, ls, d_txt,
                           None if d_txt_n is None else d_txt_n.contiguous().float())
        return d_img, d_txt, None, None


def head_apply(img_f, txt_f, logit_scale, probs: bool):
    return _HeadFn.apply(img_f, txt_f, logit_scale, probs)


class _L2NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f):
        f = f.contiguous().float()
        out = torch.empty_like(f)
        nrm = torch.empty(f.shape[0], dtype=F32, device=f.device)
        ops.l2norm_rows(f, out, nrm)
        ctx.save_for_backward(out, nrm)
        return out

    @staticmethod
    def backward(ctx, dn):
        out, nrm = ctx.saved_tensors
        # dF = (dn - n (n.dn)) / |f|: the head-gradient kernel with no logit term (Co = 1, dlog = 0)
        zero = torch.zeros(out.shape[0], 1, dtype=F32, device=out.device)
        one = torch.zeros(1, dtype=F32, device=out.device)
        dF = torch.empty_like(out)
        ops.head_feat_grad(zero, 1, 1, out[:1], out, nrm, one, dF, dn.contiguous().float())
        return dF


def l2norm_apply(f):
    return _L2NormFn.apply(f)


class _PromptTowerFn(torch.autograd.Function):
    """Prompt-tuned image tower (models/mvp_clip.py:158-175, 256-262): the frozen blocks with
    prompt tokens appended at the listed layers; gradients flow to the prompt tensors only."""

    @staticmethod
    def forward(ctx, tower, x0, n, L, training, save, layers, *prompts):
        pd = {l: p.detach().contiguous().float() for l, p in zip(layers, prompts)}
        f, c = tower.forward_embedded(x0, n, L, save, training, prompts=pd)
        ctx.tower, ctx.saved_ctx, ctx.layers = tower, c, layers
        return f

    @staticmethod
    def backward(ctx, df):
        if ctx.saved_ctx is None:
            raise RuntimeError("prompt tower forward ran without saving activations")
        pg = {}
        ctx.tower.backward(ctx.saved_ctx, df.contiguous().float(), {}, prompt_grads=pg)
        ctx.saved_ctx = None
        return (None, None, None, None, None, None, None, *[pg[l] for l in ctx.layers])


def prompt_tower_apply(tower, transformer, x0, n, L, prompts: dict, training):
    """prompts: {layer: [n, P, D]} (autograd-tracked). Returns image features [n, E]."""
    _check_frozen(tower.stack)
    layers = sorted(prompts)
    ps = [prompts[l] for l in layers]
    save = torch.is_grad_enabled() and any(p.requires_grad for p in ps)
    return _PromptTowerFn.apply(tower, x0, n, L, bool(training), save, layers, *ps)


def _deep_grad(pg, layer, shape, like):
    """Summed-over-sequences gradient of a replaced-row prompt; zero when the tower has no such
    layer (the reference's counter never reaches that prompt, maple_clip/model.py:366)."""
    g = pg.get(("R", layer))
    return g.sum(0) if g is not None else torch.zeros(shape, dtype=F32, device=like.device)


class _MapleTextFn(torch.autograd.Function):
    """MaPLe TextEncoder (models/maple.py:40-61) on the engine: the learned input embeddings
    x0 [C, L, D] and the deep text prompts replacing rows 1..n_ctx at layers 1.. (maple_clip
    model.py:381-395). Gradients: d x0 (to ctx through autograd) and the deep prompts."""

    @staticmethod
    def forward(ctx, tower, tokens, training, save, consumer, x0, *deep):
        C, L, D = x0.shape
        replace = {i + 1: (1, d.detach().float().contiguous()) for i, d in enumerate(deep)}
        f, c = tower.forward(tokens, save, training,
                             x0=x0.detach().float().reshape(C * L, D).contiguous(),
                             replace=replace)
        ctx.tower, ctx.saved_ctx, ctx.shape, ctx.n_deep = tower, c, (C, L, D), len(deep)
        ctx.deep_shapes = [tuple(d.shape) for d in deep]
        ctx.consumer = consumer
        if consumer is not None:  # read on the consumer stream (the head)
            f.record_stream(consumer)
        return f

    @staticmethod
    def backward(ctx, df):
        # autograd runs this on the forward's stream (the text stream when `consumer` is set):
        # df comes from the consumer stream, the results go back to it
        if ctx.consumer is not None:
            df.record_stream(torch.cuda.current_stream(df.device))
        pg = {}
        gx = ctx.tower.backward(ctx.saved_ctx, df.contiguous().float(), {}, prompt_grads=pg,
                                need_dx=True)
        ctx.saved_ctx = None
        d_deep = [_deep_grad(pg, i + 1, ctx.deep_shapes[i], df) for i in range(ctx.n_deep)]
        if ctx.consumer is not None:
            for t in (gx, *d_deep):
                t.record_stream(ctx.consumer)
        return (None, None, None, None, None, gx.view(*ctx.shape), *d_deep)


class _MapleImageFn(torch.autograd.Function):
    """MaPLe VisionTransformer_MaPLe.forward (maple_clip/model.py:551-590) on the engine: the
    shared visual context appended before ln_pre, deep visual prompts replacing the last n_ctx
    rows at layers 1.. (model.py:364-380)."""

    @staticmethod
    def forward(ctx, tower, img, training, save, shared, *deep):
        keep = {}
        x0, n, L = tower.embed(img, extra=shared, keep=keep if save else None)
        P = shared.shape[0]
        replace = {i + 1: (L - P, d.detach().float().contiguous()) for i, d in enumerate(deep)}
        f, c = tower.forward_embedded(x0, n, L, save, training, replace=replace)
        ctx.tower, ctx.saved_ctx, ctx.keep, ctx.P, ctx.n_deep = tower, c, keep, P, len(deep)
        ctx.deep_shapes = [tuple(d.shape) for d in deep]
        return f

    @staticmethod
    def backward(ctx, df):
        pg = {}
        gx = ctx.tower.backward(ctx.saved_ctx, df.contiguous().float(), {}, prompt_grads=pg,
                                need_dx=True)
        ctx.saved_ctx = None
        L = ctx.keep["L"]
        d_shared = ctx.tower.embed_backward(ctx.keep, gx, L - ctx.P)
        d_deep = [_deep_grad(pg, i + 1, ctx.deep_shapes[i], df) for i in range(ctx.n_deep)]
        return (None, None, None, None, d_shared, *d_deep)


def maple_text_apply(tower, tokens, x0, deep, training, consumer=None):
    """consumer: the stream that reads the features when this runs on another one (MaPLe's text
    stream); the allocator then keeps the cross-stream tensors alive for it."""
    _check_frozen(tower.stack)
    save = torch.is_grad_enabled() and (x0.requires_grad or any(d.requires_grad for d in deep))
    return _MapleTextFn.apply(tower, tokens, bool(training), save, consumer, x0, *deep)


def maple_image_apply(tower, img, shared, deep, training):
    _check_frozen(tower.stack)
    save = torch.is_grad_enabled() and (shared.requires_grad or any(d.requires_grad for d in deep))
    return _MapleImageFn.apply(tower, img, bool(training), save, shared, *deep)
