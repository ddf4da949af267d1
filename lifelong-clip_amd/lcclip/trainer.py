"""The online-CL optimizer step of methods/adapter_clip.py:49-107 (online_train) on the fused
engines, plus data-parallel replication over RCCL.

One step = image tower fwd -> text tower fwd -> normalise + logits + softmax + CE-on-probs
(fwd and bwd fused in one head kernel) -> text/image tower bwd (PEFT grads only) ->
[RCCL all-reduce of the flat PEFT-gradient buffer] -> non-finite check -> fused AdamW.

All trainable tensors live in ONE flat fp32 buffer (parameters are views into it), and so do
their gradients and the AdamW moments, so the optimizer is a single launch and the DP exchange
is a single all-reduce (1.47 MB LoRA / 7.93 MB adapter for ViT-B/16 both towers).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ops
from .adapter_clip import freeze_backbone
from .ops import F32


def remap_labels(labels, class_list=None):
    """methods/adapter_clip.py:53-61, 75-76 with visible_classes='batch': the class list is the
    distinct labels in first-seen order and y becomes an index into it. Under DP every rank
    passes the GLOBAL batch labels so all ranks agree on the logit columns."""
    class_list = [] if class_list is None else list(class_list)
    ys = labels.tolist()
    for y in ys:
        if y not in class_list:
            class_list.append(y)
    return torch.tensor([class_list.index(y) for y in ys], dtype=torch.long), class_list


class OnlineTrainer:
    def __init__(self, adapter_clip, lr=5e-4, weight_decay=1e-5, betas=(0.9, 0.999), eps=1e-8,
                 process_group=None, distributed=None):
        self.wrapper = adapter_clip
        self.clip = adapter_clip.model
        freeze_backbone(self.wrapper)
        self.img = self.clip.visual.tower
        self.txt = self.clip.text_tower
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.group = process_group
        self.distributed = (dist.is_available() and dist.is_initialized()) if distributed is None else distributed
        params = self.img.stack.trainable_params() + self.txt.stack.trainable_params()
        dev = self.clip.logit_scale.device
        n = sum(p.numel() for p in params)
        self.numel = n
        self.flat_p = torch.empty(n, dtype=F32, device=dev)
        self.flat_g = torch.zeros(n, dtype=F32, device=dev)
        self.m = torch.zeros(n, dtype=F32, device=dev)
        self.v = torch.zeros(n, dtype=F32, device=dev)
        self.grads = {}
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                self.flat_p[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat_p[off:off + k].view_as(p)
                self.grads[p] = self.flat_g[off:off + k].view_as(p)
                off += k
        self.params = params
        self.skip = torch.zeros(1, dtype=torch.int32, device=dev)
        self.step_count = 0
        self.logit_scale = self.clip.logit_scale.detach().reshape(1)

    def reset_optimizer(self):
        """online_before_task rebuilds AdamW per task (methods/adapter_clip.py:127, Q14)."""
        self.m.zero_()
        self.v.zero_()
        self.step_count = 0

    def forward_backward(self, images, labels, tokens):
        """Everything but the optimizer update. Returns (loss[1], probs[B,C])."""
        dev = self.flat_g.device
        self.flat_g.zero_()
        f_i, ci = self.img.forward(images, save=True, training=True)
        f_t, ct = self.txt.forward(tokens, save=True, training=True)
        B, E = f_i.shape
        C = f_t.shape[0]
        img_n = torch.empty_like(f_i)
        txt_n = torch.empty_like(f_t)
        ni = torch.empty(B, dtype=F32, device=dev)
        nt = torch.empty(C, dtype=F32, device=dev)
        ops.l2norm_rows(f_i, img_n, ni)
        ops.l2norm_rows(f_t, txt_n, nt)
        probs = torch.empty(B, C, dtype=F32, device=dev)
        dlog = torch.empty(B, C, dtype=F32, device=dev)
        loss = torch.zeros(1, dtype=F32, device=dev)
        labels = labels.to(dev, torch.int64).contiguous()
        ops.clip_head(img_n, txt_n, self.logit_scale, labels, probs, dlog, loss)
        d_i = torch.empty_like(f_i)
        d_t = torch.empty_like(f_t)
        ops.head_feat_grad(dlog, C, 1, txt_n, img_n, ni, self.logit_scale, d_i)
        ops.head_feat_grad(dlog, 1, C, img_n, txt_n, nt, self.logit_scale, d_t)
        if ct is not None and self.txt.stack.trainable_params():
            self.txt.backward(ct, d_t, self.grads)
        if self.img.stack.trainable_params():
            self.img.backward(ci, d_i, self.grads)
        return loss, probs

    def all_reduce_grads(self):
        if self.distributed:
            dist.all_reduce(self.flat_g, op=dist.ReduceOp.AVG, group=self.group)

    def optimizer_step(self):
        self.step_count += 1
        self.skip.zero_()
        ops.check_finite(self.flat_g, self.skip)
        b1, b2 = self.betas
        ops.adamw(self.flat_p, self.flat_g, self.m, self.v, self.lr, b1, b2, self.eps, self.wd,
                  self.step_count, self.skip)

    def step(self, images, labels, tokens):
        loss, probs = self.forward_backward(images, labels, tokens)
        self.all_reduce_grads()
        self.optimizer_step()
        return loss, probs
