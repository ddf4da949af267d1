"""Data-parallel exchange of the online step, one process per GPU.

The reference replicates the model with nn.DataParallel and computes ONE loss over the gathered
global batch (methods/adapter_clip.py:84-89, _trainer.py:168); the backbone is frozen, the loss
is per-image CE over class logits, so images shard along the batch with no data-path collective.
What remains is:

  * replicas: the reference's DataParallel re-broadcasts every parameter and buffer from GPU 0
    on every forward (replicate -> broadcast_coalesced, _trainer.py:167-168). Here the
    weights are replicated ONCE, when the trainer is built: rank 0's frozen backbone, buffers and
    flat PEFT parameters are broadcast to every rank (broadcast_from_root), and from then on the
    ranks stay identical because they apply the same averaged gradients with the same AdamW.

  * PEFT gradients: averaged over ranks. They live in one flat fp32 buffer; per-layer-group
    buckets are all-reduced asynchronously as soon as backward has finished those layers, so
    the exchange overlaps the rest of backward (RCCL runs on its own stream; on gloo the same
    calls run on the CPU for the tests). SUM on the wire, one 1/world scale at the end (gloo has
    no AVG).
  * text prompts: every rank needs the features of ALL C prompts (the logit columns), but the
    text tower is not replicated: rank r encodes prompts [r*per, (r+1)*per) (the list padded to
    per*world by repeating the last prompt), the feature rows are all-gathered, and dL/dT from
    every rank's images is all-reduced (SUM) before each rank backpropagates its own slice.
    Because dT is summed, a rank's text gradients come out world x its slice's share; the final
    1/world scale of the flat buffer then leaves exactly the sum of the slices — the gradient of
    the global-mean loss.
  * labels / class list: every rank passes the GLOBAL batch labels to remap_labels so the logit
    columns agree (the reference MVP trainer all-gathers them, methods/mvp_clip.py:305-313).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class DataParallel:
    """Rank bookkeeping + the three exchanges. world == 1 makes every call a no-op, unless the
    collectives are forced (env LCCLIP_DP_FORCE=1 with an initialised process group: the same
    calls run on a one-rank group, so the RCCL path executes on a one-GPU box)."""

    def __init__(self, group=None, enabled=None):
        import os
        on = dist.is_available() and dist.is_initialized()
        self.enabled = on if enabled is None else (enabled and on)
        self.group = group
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.rank = dist.get_rank(group) if self.enabled else 0
        self.active = self.world > 1 or (self.enabled and os.environ.get("LCCLIP_DP_FORCE") == "1")
        self._works = []

    # ---------------------------------------------------------------- replication
    def root_rank(self):
        """The global rank of the group's rank 0."""
        if self.group is None:
            return 0
        return dist.get_global_rank(self.group, 0)

    def broadcast_from_root(self, tensors, bucket_bytes=64 << 20):
        """Overwrite `tensors` (in place) with rank 0's values, once. Same-dtype tensors on one
        device go in flattened buckets of about `bucket_bytes` (a few large broadcasts instead of
        one per tensor: the ViT-B/16 backbone is ~300 tensors, 600 MB in f32)."""
        if not self.active:
            return
        src = self.root_rank()
        groups = {}
        for t in tensors:
            groups.setdefault((t.dtype, t.device), []).append(t)
        for (dtype, device), ts in groups.items():
            bucket, nbytes = [], 0
            for t in ts + [None]:
                if t is not None:
                    bucket.append(t)
                    nbytes += t.numel() * t.element_size()
                if bucket and (t is None or nbytes >= bucket_bytes):
                    flat = torch.cat([b.detach().reshape(-1) for b in bucket])
                    dist.broadcast(flat, src=src, group=self.group)
                    off = 0
                    with torch.no_grad():
                        for b in bucket:
                            b.copy_(flat[off:off + b.numel()].view_as(b))
                            off += b.numel()
                    bucket, nbytes = [], 0

    # ---------------------------------------------------------------- prompt sharding
    def prompt_slice(self, C: int):
        """(lo, hi, per): this rank's rows of the padded prompt list."""
        per = -(-C // self.world)
        lo = self.rank * per
        return lo, lo + per, per

    def shard_tokens(self, tokens):
        C = tokens.shape[0]
        lo, hi, per = self.prompt_slice(C)
        pad = per * self.world - C
        if pad:
            tokens = torch.cat([tokens, tokens[-1:].expand(pad, -1)], 0)
        return tokens[lo:hi].contiguous()

    def gather_rows(self, rows, C: int):
        """All-gather the per-rank [per, E] feature slices into [C, E] (padding dropped)."""
        if not self.active:
            return rows[:C]
        parts = [torch.empty_like(rows) for _ in range(self.world)]
        dist.all_gather(parts, rows.contiguous(), group=self.group)
        return torch.cat(parts, 0)[:C]

    def sum_async(self, t):
        """Asynchronous in-place SUM all-reduce; returns a handle with .wait() (or None)."""
        if not self.active:
            return None
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    # ---------------------------------------------------------------- gradient buckets
    def launch_bucket(self, flat, lo: int, hi: int):
        if self.active and hi > lo:
            self._works.append(self.sum_async(flat[lo:hi]))

    def finish_buckets(self, flat):
        """Wait for every bucket and turn the sums into means."""
        if not self.active:
            return
        for w in self._works:
            w.wait()
        self._works.clear()
        flat.mul_(1.0 / self.world)


class ModuleDataParallel:
    """One process per GPU for the autograd model surfaces (CLIP_MVP, BASELINE config 3; MaPLe,
    config 5; AdapterCLIP's module path): the reference's single-process nn.DataParallel
    (methods/_trainer.py:167-168) as one rank per GPU over RCCL.

      * replicas: rank 0's parameters and buffers are broadcast once, at construction (the
        one-time form of DataParallel's per-step replicate);
      * the exposed class list: every rank contributes the classes of its share of the batch
        and all ranks take the same merged list, in rank order, first occurrence kept — what the
        reference's MVP trainer does with all_gather (methods/mvp_clip.py:300-313), so the logit
        columns agree;
      * gradients: after backward, the trainable parameters' gradients (MVP: key, mask,
        g_prompts, e_prompts; MaPLe: the prompt learner) are all-reduced in flat buckets,
        launched asynchronously one after another, and averaged — with equal per-rank batches
        the gradient of the global-mean loss, which is what the reference's one loss over the
        gathered outputs gives;
      * per-batch statistics the modules keep (CLIP_MVP.count, mvp_clip.py:239-241) are summed
        over ranks through `all_sum`, so every replica counts the global batch.
    world == 1 (without LCCLIP_DP_FORCE) makes every call a no-op."""

    def __init__(self, module, group=None, enabled=None, bucket_bytes=25 << 20):
        self.module = module
        self.dp = DataParallel(group, enabled)
        self.bucket_bytes = int(bucket_bytes)
        self.active = self.dp.active
        if self.active:
            tensors = [p.data for p in module.parameters()]
            tensors += [b for b in module.buffers()
                        if b.numel() and (b.is_floating_point() or b.dtype == torch.int64)]
            self.dp.broadcast_from_root(tensors)
            _invalidate_staging(module)
        module._dp = self

    @property
    def world(self):
        return self.dp.world

    @property
    def rank(self):
        return self.dp.rank

    def exposed_classes(self, local_classes):
        """The global batch's class list from every rank's list (methods/mvp_clip.py:300-313)."""
        local = [int(c) for c in local_classes]
        if not self.active:
            out = []
        else:
            parts = [None] * self.dp.world
            dist.all_gather_object(parts, local, group=self.dp.group)
            local = [c for part in parts for c in part]
            out = []
        for c in local:
            if c not in out:
                out.append(c)
        return out

    def all_sum(self, t):
        """In-place SUM over ranks (blocking for the caller's stream)."""
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.dp.group)
        return t

    def sync_grads(self):
        """Average the trainable parameters' gradients over ranks (call after backward, before
        the optimizer step)."""
        if not self.active:
            return
        params = [p for p in self.module.parameters() if p.requires_grad]
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        groups = {}
        for p in params:
            groups.setdefault((p.grad.dtype, p.grad.device), []).append(p)
        works = []
        for ps in groups.values():
            bucket, nbytes = [], 0
            for p in ps + [None]:
                if p is not None:
                    bucket.append(p)
                    nbytes += p.grad.numel() * p.grad.element_size()
                if bucket and (p is None or nbytes >= self.bucket_bytes):
                    flat = torch.cat([q.grad.reshape(-1) for q in bucket])
                    works.append((dist.all_reduce(flat, op=dist.ReduceOp.SUM,
                                                  group=self.dp.group, async_op=True),
                                  flat, bucket))
                    bucket, nbytes = [], 0
        inv = 1.0 / self.dp.world
        for w, flat, bucket in works:
            w.wait()
            flat.mul_(inv)
            off = 0
            for q in bucket:
                q.grad.copy_(flat[off:off + q.numel()].view_as(q.grad))
                off += q.numel()


def _invalidate_staging(module):
    """Drop every staged weight image under `module` (the tower engines re-stage from the
    broadcast values; in-place collectives do not bump the tensors' version counters)."""
    for m in module.modules():
        eng = getattr(m, "_engine", None)
        if eng is not None:
            eng.invalidate_all()
        for name in ("_tower", "_text_tower"):
            t = getattr(m, name, None)
            if t is not None:
                t._key = None
        cache = getattr(m, "_txt_cache", None)
        if cache is not None:
            cache.clear()


def layer_ranges(stack, base: int = 0):
    """[(lo, hi)] offsets of each block's PEFT parameters inside a flat buffer whose layout is
    stack.trainable_params() in order, starting at `base`."""
    out = []
    off = base
    for b in stack.blocks:
        n = sum(p.numel() for p in b.peft_parameters())
        out.append((off, off + n))
        off += n
    return out
