"""The online-CL optimizer step of methods/adapter_clip.py:49-107 (online_train) on the fused
engines, plus data-parallel replication over RCCL.

One step = image tower fwd -> text tower fwd (this rank's prompt slice under DP) -> normalise
+ logits + softmax + CE-on-probs (fwd and bwd fused in one head kernel) -> image tower bwd
(PEFT grads only; per-layer-group RCCL buckets launched as layers finish) -> text tower bwd ->
non-finite check -> fused AdamW. The DP exchange is described in dp.py.

All trainable tensors live in ONE flat fp32 buffer (parameters are views into it), and so do
their gradients and the AdamW moments, so the optimizer is a single launch and the DP exchange
is a single all-reduce (1.47 MB LoRA / 7.93 MB adapter for ViT-B/16 both towers).
"""
from __future__ import annotations

import os

import torch

from . import ops
from .dp import DataParallel, layer_ranges
from .adapter_clip import freeze_backbone
from .ops import F32
from .textcache import TokenFeatureCache


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


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
                 process_group=None, distributed=None, shard_text=True, bucket_layers=4,
                 overlap_text=True, overlap_grads=True, side_cus=None):
        self.wrapper = adapter_clip
        self.clip = adapter_clip.model
        freeze_backbone(self.wrapper)
        self.img = self.clip.visual.tower
        self.txt = self.clip.text_tower
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.dp = DataParallel(process_group, distributed)
        self.distributed = self.dp.active
        self.shard_text = shard_text and self.distributed
        self.bucket_layers = max(1, int(bucket_layers))
        img_params = self.img.stack.trainable_params()
        params = img_params + self.txt.stack.trainable_params()
        n_img = sum(p.numel() for p in img_params)
        self.img_ranges = layer_ranges(self.img.stack) if img_params else []
        self.txt_range = (n_img, sum(p.numel() for p in params))
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
        if self.distributed:
            self.replicate()
        self.skip = torch.zeros(1, dtype=torch.int32, device=dev)
        # AdamW's step (bias correction) lives on the device and advances only for applied
        # updates; step_count counts optimizer_step() calls, skipped ones included
        self.adam_step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.step_count = 0
        self.graph = None
        self.overlap_text = bool(overlap_text)
        self.overlap_grads = bool(overlap_grads)
        self._side = None
        self._gstream = None
        # side streams confined to a CU subset: (count, stride, first) or None (every CU);
        # LCCLIP_SIDE_CUS="count[,stride[,first]]" for A/Bs
        env = os.environ.get("LCCLIP_SIDE_CUS")
        if side_cus is None and env:
            side_cus = tuple(int(v) for v in env.split(","))
        self.side_cus = None if side_cus is None else (tuple(side_cus) + (1, 0)[len(side_cus) - 1:])[:3]
        self._masked = []
        self._txt_cache = TokenFeatureCache()
        self.logit_scale = self.clip.logit_scale.detach().reshape(1)

    def replicate(self):
        """Make every rank's model rank 0's, once (the one-time form of nn.DataParallel's
        per-step replicate, methods/_trainer.py:167-168): the frozen backbone parameters, the
        buffers (text_tokens included) and the flat PEFT parameter buffer are broadcast from
        rank 0, and every staged weight image is dropped so the next forward re-stages from the
        broadcast values."""
        peft = {id(p) for p in self.params}
        frozen = [p for p in self.wrapper.parameters() if id(p) not in peft]
        bufs = [b for b in self.wrapper.buffers() if b.is_floating_point() or b.dtype == torch.int64]
        self.dp.broadcast_from_root([self.flat_p] + [p.data for p in frozen] + bufs)
        for st in (self.img.stack, self.txt.stack):
            st.invalidate_all()
        self.img._key = None
        self.txt._key = None

    def reset_optimizer(self):
        """online_before_task rebuilds AdamW per task (methods/adapter_clip.py:127, Q14)."""
        self.m.zero_()
        self.v.zero_()
        self.step_count = 0
        self.adam_step.zero_()

    def forward_backward(self, images, labels, tokens):
        """Everything but the optimizer update. Returns (loss[1], probs[B,C]).

        The text tower (C prompts x 77 tokens: small, latency-bound launches) runs on a side HIP
        stream concurrently with the image tower, forward and backward; the two meet at the
        logit head and again before the gradient exchange/optimizer (`overlap_text`)."""
        dev = self.flat_g.device
        self.flat_g.zero_()
        dp = self.dp
        C = tokens.shape[0]
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev)
        if side is not None:
            side.wait_stream(main)
        if not labels.is_cuda and labels.numel() and (int(labels.min()) < 0 or int(labels.max()) >= C):
            raise ValueError(f"labels must index the {C} prompts (remap them against the global "
                             "class list, trainer.remap_labels)")
        tok_in = dp.shard_tokens(tokens) if self.shard_text else tokens
        cached = self._cached_text(tokens)
        if cached is None:
            train_t = bool(self.txt.stack.trainable_params())
            with torch.cuda.stream(side) if side is not None else _nullctx():
                f_t, ct = self.txt.forward(tok_in, save=train_t, training=True)
        f_i, ci = self.img.forward(images, save=True, training=True)
        if side is not None:
            main.wait_stream(side)
        if cached is not None:
            f_t, ct = cached, None
        else:
            if self.shard_text:
                f_t = dp.gather_rows(f_t, C).contiguous()
            self._store_text(tokens, f_t)
        B, E = f_i.shape
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
        lo, hi, per = dp.prompt_slice(C) if self.shard_text else (0, C, C)
        d_tp = torch.zeros(per * dp.world if self.shard_text else C, E, dtype=F32, device=dev)
        ops.head_feat_grad(dlog, C, 1, txt_n, img_n, ni, self.logit_scale, d_i)
        train_txt = ct is not None and bool(self.txt.stack.trainable_params())
        # dL/dT (a sum over the batch per prompt) is only needed by the text backward: it is
        # computed on the text stream, off the image chain, and (sharded text) all-reduced from
        # there, so RCCL's stream follows the text stream and only the text backward waits for it
        if train_txt:
            if side is not None:
                side.wait_stream(main)
            with torch.cuda.stream(side) if side is not None else _nullctx():
                ops.head_feat_grad(dlog, 1, C, img_n, txt_n, nt, self.logit_scale, d_tp[:C])
                w_dt = dp.sum_async(d_tp) if self.shard_text else None
                if w_dt is not None:
                    w_dt.wait()  # the current (text) stream waits for the dL/dT all-reduce
                self.txt.backward(ct, d_tp[lo:hi].contiguous(), self.grads)
        if self.img.stack.trainable_params():
            self.img.backward(ci, d_i, self.grads, on_layer=self._img_bucket_hook(),
                              grad_stream=self._grad_stream(dev))
        if side is not None:
            main.wait_stream(side)
        dp.launch_bucket(self.flat_g, *self.txt_range)
        return loss, probs

    # frozen text tower (peft_encoder 'image' / 'none'): features cached per token content
    # (lcclip.textcache: rank-invariant hit decision, no stale hits on reused storage)
    def _weights_key(self):
        c = self.clip
        return (tuple(p._version for p in c.transformer.parameters()),
                c.token_embedding.weight._version, c.text_projection._version,
                c.ln_final.weight._version)

    def _cacheable(self):
        return not (self.txt.stack.trainable_params() or torch.cuda.is_current_stream_capturing())

    def _cached_text(self, tokens):
        if not self._cacheable():
            return None
        return self._txt_cache.get(tokens, self._weights_key())

    def _store_text(self, tokens, f_t):
        if self._cacheable():
            self._txt_cache.put(tokens, self._weights_key(), f_t)
        else:
            self._txt_cache.clear()

    def _grad_stream(self, dev):
        if not self.overlap_grads:
            return None
        if self._merge_side_streams():
            side = self._side_stream(dev)
            if side is not None:
                return side
        if self._gstream is None:
            self._gstream = self._new_stream(dev)
        return self._gstream

    def _new_stream(self, dev):
        if self.side_cus is None:
            return torch.cuda.Stream(device=dev)
        count, stride, first = self.side_cus
        ms = ops.CUMaskedStream(dev, count, stride, first)
        self._masked.append(ms)  # owns the HIP stream
        return ms.stream

    def _merge_side_streams(self):
        """One side stream for the text tower AND the PEFT weight gradients when the process
        group is up and HIP has few hardware queues. HIP maps streams onto GPU_MAX_HW_QUEUES
        queues (default 4; the value exported when lcclip was imported, which is the one HIP read if
        it initialised after that); main + text + weight-gradient streams + RCCL's own is one stream too
        many, and the side streams then land on the main stream's queue and stop overlapping it
        (r2: 7308 vs 8172 img/s at N = 1 with the exchange forced on). Sharing one side stream
        keeps every stream on its own queue at the default. LCCLIP_SIDE_STREAMS=1|2 forces it."""
        force = os.environ.get("LCCLIP_SIDE_STREAMS")
        if force in ("1", "2"):
            return force == "1"
        from . import HW_QUEUES_AT_IMPORT
        try:
            queues = int(HW_QUEUES_AT_IMPORT or "4")
        except ValueError:
            queues = 4
        return self.distributed and queues < 6

    def _side_stream(self, dev):
        if not self.overlap_text:
            return None
        if self._side is None:
            self._side = self._new_stream(dev)
        return self._side

    def _img_bucket_hook(self):
        """Launch the all-reduce of image layers [li, prev) every bucket_layers layers."""
        if not self.distributed:
            return None
        state = {"hi": len(self.img_ranges)}

        def hook(li):
            if li % self.bucket_layers == 0:
                lo_r = self.img_ranges[li][0]
                hi_r = self.img_ranges[state["hi"] - 1][1]
                gs = getattr(self.img.stack, "_gs", None)
                if gs is None:
                    self.dp.launch_bucket(self.flat_g, lo_r, hi_r)
                else:
                    # the bucket's gradients come from both streams: the gradient stream waits
                    # for the main one (never the reverse: the main chain keeps running) and the
                    # all-reduce is issued from it, so RCCL's stream follows both
                    gs.wait_stream(torch.cuda.current_stream(gs.device))
                    with torch.cuda.stream(gs):
                        self.dp.launch_bucket(self.flat_g, lo_r, hi_r)
                state["hi"] = li
        return hook

    def all_reduce_grads(self):
        """Wait for the bucketed exchange launched during backward; grads become rank means."""
        self.dp.finish_buckets(self.flat_g)

    def optimizer_step(self):
        self.step_count += 1
        self._update()

    def _update(self):
        """Non-finite check -> AdamW step counter (unless skipped) -> fused AdamW, all on the
        device (no host sync)."""
        self.skip.zero_()
        ops.check_finite(self.flat_g, self.skip)
        ops.adam_step_advance(self.adam_step, self.skip)
        b1, b2 = self.betas
        ops.adamw(self.flat_p, self.flat_g, self.m, self.v, self.lr, b1, b2, self.eps, self.wd, 1,
                  self.skip, step_dev=self.adam_step)
        # the update bypassed torch's version counters: re-stage the PEFT-derived weights
        self.img.stack.invalidate_peft()
        self.txt.stack.invalidate_peft()

    def step(self, images, labels, tokens):
        if self.graph is not None:
            return self._replay(images, labels, tokens)
        return self.eager_step(images, labels, tokens)

    def eager_step(self, images, labels, tokens):
        """One step launched op by op (also available when a graph is active, e.g. to time the
        individual kernels)."""
        loss, probs = self.forward_backward(images, labels, tokens)
        self.all_reduce_grads()
        self.optimizer_step()
        return loss, probs

    # ------------------------------------------------------------------ HIP graph replay
    def enable_graph(self, images, labels, tokens, warmup=2):
        """Capture one whole step (fwd, head, bwd, non-finite check, AdamW) as a HIP graph and
        replay it from then on: the ~650 launches of a step leave the host once, with no
        inter-kernel gaps. Shapes are fixed at capture; `images` / `labels` / `tokens` become the
        graph's input buffers (a later step() with other tensors copies into them). The dropout
        masks and AdamW's bias correction read device-side counters that the graph advances on
        every replay. Single process only: under torch.distributed the step stays eager.
        step() then returns fresh copies of the graph's (loss, probs) buffers.
        Returns True when the graph is active."""
        if self.distributed:
            return False
        dev = self.flat_p.device
        self._gx = images
        self._gy = labels.to(dev, torch.int64).contiguous()
        self._gt = tokens.contiguous()
        self.ctr = torch.zeros(1, dtype=torch.int64, device=dev)  # dropout RNG epoch
        for st in (self.img.stack, self.txt.stack):
            st.seed_dev = self.ctr[0:1]
        # warm-up steps (allocator, lazy staging) must not change the model: snapshot + restore
        state = (self.flat_p, self.m, self.v, self.ctr, self.adam_step)
        snap = [t.clone() for t in state]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._graph_body()
        torch.cuda.current_stream(dev).wait_stream(side)
        for t, c in zip(state, snap):
            t.copy_(c)
        self.img.stack.invalidate_peft()
        self.txt.stack.invalidate_peft()
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._g_out = self._graph_body()
        self.graph = g
        return True

    def _graph_body(self):
        ops.counter_add(self.ctr, 1)
        loss, probs = self.forward_backward(self._gx, self._gy, self._gt)
        self._update()
        # captured merges must re-run on every replay: stage again inside the next capture/run
        self.img.stack.invalidate_peft()
        self.txt.stack.invalidate_peft()
        return loss, probs

    def _replay(self, images, labels, tokens):
        if images.data_ptr() != self._gx.data_ptr():
            self._gx.copy_(images)
        if labels.data_ptr() != self._gy.data_ptr():
            self._gy.copy_(labels.to(self._gy.device, torch.int64))
        if tokens.data_ptr() != self._gt.data_ptr():
            self._gt.copy_(tokens)
        self.graph.replay()
        self.step_count += 1
        # the captured outputs are overwritten by the next replay: hand out copies
        return tuple(t.clone() for t in self._g_out)
