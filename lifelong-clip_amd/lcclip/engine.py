"""Tower engines: the fused forward/backward of a stack of CLIP residual blocks and of the two
encoders, entirely through liblcclip.so kernels.

Reference semantics (qcNPU/LifeLong-CLIP):
  block        models/clip/model.py:233-236 (vanilla / LoRA), :439-442 (adapter, Q6)
  LoRA MHA     models/clip/lora.py:832-1074
  adapter      models/clip/adapter.py:53-72
  image tower  models/clip/model.py:755-787 (Q1: blocks called as blk(x))
  text tower   models/clip/model.py:941-956

Data layout in HBM (rows = sequence * L tokens, batch-major; the reference's sequence-first
layout is internal and not observable):
  residual stream   f32  [rows, D]   one buffer per sub-block output (kept for LN backward)
  LN outputs        bf16 [rows, D]   transient unless a LoRA in-proj needs them for dA
  qkv               bf16 [rows, 3D]  kept (attention backward)
  attention out O   bf16 [rows, D]   kept; lse f32 [seq*H, L]
  MLP pre-activation bf16 [rows, 4D] kept (QuickGELU backward); GELU output transient
  adapter input z   bf16 [rows, D], bottleneck h bf16 [rows, 64]  kept
Frozen weights are staged once as bf16 in both [out,in] and [in,out] layouts (forward and dX
GEMMs are both A @ B^T); LoRA blocks re-merge W + s*B@A into those buffers each step.
The backbone is frozen: backward produces input gradients and PEFT parameter gradients only.

precision='fp8' (BlockStack attribute; MaPLe's image tower under BASELINE config 5): the QKV,
c_fc and c_proj GEMMs, forward and input-gradient, run as block-scaled e4m3 GEMMs on the fp8
MFMA (ops.gemm_nt_fp8). Their frozen weights are quantised once per checkpoint in both layouts
(from the f32 master, or from the bf16 LoRA merge), their activation / gradient operands at the
call; out-projection, attention, LayerNorm and the residual stream stay as in bf16 mode.
"""
from __future__ import annotations

import itertools
import os

import torch

from . import ops
from .ops import BF16, F16, F32, EPI_BF16, EPI_F32, EPI_GELU, EPI_GELU_D, EPI_MUL, EPI_RESID
from .ops import EPI_RESID16
from .ops import EPI_GELU_D_Q8, EPI_MUL_Q8

_seed_counter = itertools.count(1)


def _empty(shape, dtype, dev):
    """(dtype None: a buffer that is not kept -> None)"""
    return None if dtype is None else torch.empty(shape, dtype=dtype, device=dev)


def _rows(t, n):
    return None if t is None else t[:n]


def _key(*tensors):
    return tuple((t.data_ptr(), t._version) for t in tensors if t is not None)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class StagedBlock:
    """bf16 device copies of one block's GEMM weights (both layouts)."""

    def __init__(self):
        self.frozen_key = None
        self.peft_key = None
        self.merge_epoch = 0  # advanced on every LoRA re-merge (part of the fp8 staging key)


class BlockStack:
    """Engine for `Transformer.resblocks` (model.py:639-686): a list of block modules sharing
    width, heads, mask and PEFT variant."""

    def __init__(self, blocks, n_head: int, causal: bool, variant: str):
        self.blocks = list(blocks)
        self.n_head = n_head
        self.causal = bool(causal)
        self.variant = variant  # 'vanilla' | 'lora' | 'adapter'
        self.staged = [StagedBlock() for _ in self.blocks]
        # optional int64 device tensor: RNG epoch added to every dropout seed (graph replay)
        self.seed_dev = None
        self.precision = "bf16"  # 'bf16' | 'fp8' (QKV / c_fc / c_proj on the fp8 MFMA)
        self.dt = BF16  # 16-bit storage of activations, gradients and staged weights

    def set_storage(self, dtype):
        """16-bit storage type of the stack: torch.bfloat16 (default) or torch.float16 (IEEE
        half, the reference's autocast dtype: every kernel of the stack then runs its _f16 entry
        point, include/lc_clip.h). The staged weights are re-staged in the new type."""
        if dtype not in (BF16, F16):
            raise ValueError("storage must be torch.bfloat16 or torch.float16")
        if dtype == F16 and self.precision != "bf16":
            raise ValueError("float16 storage is not combined with fp8 GEMMs")
        if dtype != self.dt:
            self.dt = dtype
            for st in self.staged:
                st.frozen_key = None
                st.peft_key = None
                for name in ("lora_in", "lora_out"):
                    st.__dict__.pop(name, None)
        return self

    # ------------------------------------------------------------------ weight staging
    def trainable_params(self):
        out = []
        for b in self.blocks:
            out.extend(b.peft_parameters())
        return out

    def backbone_params(self):
        out = []
        for b in self.blocks:
            out.extend(b.backbone_parameters())
        return out

    def invalidate_peft(self):
        """Forget the staged PEFT-derived weights (LoRA merges, adapter bf16 copies). Needed after
        any update that bypasses torch's version counters (the fused AdamW writes the flat
        parameter buffer through the C ABI)."""
        for st in self.staged:
            st.peft_key = None

    def invalidate_all(self):
        """Forget every staged weight image, frozen ones included (their source tensors were
        overwritten in place without a version bump, e.g. by a broadcast)."""
        for st in self.staged:
            st.frozen_key = None
            st.peft_key = None
            st.q_key = None

    def stage(self):
        casts, merges = [], []
        for blk, st in zip(self.blocks, self.staged):
            attn, mlp = blk.attn, blk.mlp
            fkey = _key(attn.in_proj_weight, attn.out_proj.weight, mlp.c_fc.weight, mlp.c_proj.weight)
            if fkey != st.frozen_key:
                dev = attn.in_proj_weight.device
                D = attn.in_proj_weight.shape[1]
                st.wqkv = _empty((3 * D, D), self.dt, dev)
                st.wqkvT = _empty((D, 3 * D), self.dt, dev)
                st.wo = _empty((D, D), self.dt, dev)
                st.woT = _empty((D, D), self.dt, dev)
                st.wfc = _empty((4 * D, D), self.dt, dev)
                st.wfcT = _empty((D, 4 * D), self.dt, dev)
                st.wpr = _empty((D, 4 * D), self.dt, dev)
                st.wprT = _empty((4 * D, D), self.dt, dev)
                ops.merge_weight(mlp.c_fc.weight.detach(), None, None, 0.0, st.wfc, st.wfcT)
                ops.merge_weight(mlp.c_proj.weight.detach(), None, None, 0.0, st.wpr, st.wprT)
                if self.variant != "lora":
                    ops.merge_weight(attn.in_proj_weight.detach(), None, None, 0.0, st.wqkv, st.wqkvT)
                    ops.merge_weight(attn.out_proj.weight.detach(), None, None, 0.0, st.wo, st.woT)
                st.frozen_key = fkey
                st.peft_key = None
            if self.variant == "lora":
                pkey = _key(attn.in_proj_weight_lora_A, attn.in_proj_weight_lora_B,
                            attn.out_proj.lora_A, attn.out_proj.lora_B) + fkey
                if pkey != st.peft_key:
                    s = attn.scaling
                    merges.append((attn.in_proj_weight.detach(), attn.in_proj_weight_lora_A.detach(),
                                   attn.in_proj_weight_lora_B.detach(), s, st.wqkv, st.wqkvT))
                    merges.append((attn.out_proj.weight.detach(), attn.out_proj.lora_A.detach(),
                                   attn.out_proj.lora_B.detach(), s, st.wo, st.woT))
                    # bf16 A and B^T zero-padded to 64 rows: operands of the LoRA-gradient GEMMs
                    st.lora_in = self._stage_lora(st, "lora_in", attn.in_proj_weight_lora_A,
                                                  attn.in_proj_weight_lora_B, merges)
                    st.lora_out = self._stage_lora(st, "lora_out", attn.out_proj.lora_A,
                                                   attn.out_proj.lora_B, merges)
                    st.peft_key = pkey
                    # the fused AdamW bypasses the version counters, so the re-merged weights can
                    # carry the same pkey as before: the epoch is what tells _stage_fp8 to re-quantise
                    st.merge_epoch += 1
            elif self.variant == "adapter":
                ad = blk.adaptmlp
                pkey = _key(ad.down_proj.weight, ad.up_proj.weight)
                if pkey != st.peft_key:
                    dev = ad.down_proj.weight.device
                    D = ad.down_proj.weight.shape[1]
                    H = ad.down_proj.weight.shape[0]
                    st.wd = _empty((H, D), self.dt, dev)
                    st.wdT = _empty((D, H), self.dt, dev)
                    st.wu = _empty((D, H), self.dt, dev)
                    st.wuT = _empty((H, D), self.dt, dev)
                    casts.append((ad.down_proj.weight.detach(), st.wd, st.wdT))
                    casts.append((ad.up_proj.weight.detach(), st.wu, st.wuT))
                    st.peft_key = pkey
        # the PEFT weights of every block change at each optimizer step: one launch for all
        # (LoRA: 6 merges / casts per block, a launch per CAST_MAX items)
        if casts:
            ops.cast_weights(casts)
        if merges and self.MERGE_BATCH:
            ops.merge_weights(merges)
        for item in (merges if not self.MERGE_BATCH else ()):
            ops.merge_weight(*item)
        if self.precision == "fp8":
            self._stage_fp8()

    # frozen GEMM weights quantised to the fp8 operand format, both layouts
    FP8_WEIGHTS = ("wqkv", "wqkvT", "wfc", "wfcT", "wpr", "wprT")

    def _stage_fp8(self):
        for blk, st in zip(self.blocks, self.staged):
            D = blk.attn.in_proj_weight.shape[1]
            if D % 256:
                raise ValueError(f"precision='fp8' needs a width that is a multiple of 256 (got {D}): "
                                 "the fp8 GEMM tiles N in 256-column blocks")
            key = (st.frozen_key, st.peft_key, st.merge_epoch)
            if getattr(st, "q_key", None) == key:
                continue
            attn, mlp = blk.attn, blk.mlp
            if self.variant == "lora":  # the per-step merged weights (bf16, both layouts)
                src = {"wqkv": (st.wqkv, False), "wqkvT": (st.wqkvT, False)}
            else:
                w = attn.in_proj_weight.detach()
                src = {"wqkv": (w, False), "wqkvT": (w, True)}
            wf, wp = mlp.c_fc.weight.detach(), mlp.c_proj.weight.detach()
            src.update(wfc=(wf, False), wfcT=(wf, True), wpr=(wp, False), wprT=(wp, True))
            st.q = {name: ops.quant_fp8(t, transpose=tr) for name, (t, tr) in src.items()}
            st.q_key = key

    # fp8 mode: the c_fc forward and c_proj input-gradient epilogues (EPI_GELU_D_Q8 /
    # EPI_MUL_Q8), the ln_1 / ln_2 forwards and the attention backward write their result
    # straight in the fp8 operand format of the GEMM that consumes it instead of bf16 + a
    # quant_fp8 pass (the same codes). LCCLIP_FP8_FUSE for A/Bs: 0 none, 1 the GEMM epilogues,
    # 2 + LayerNorm, 3 + attention backward, 4 (default) + ln_1's backward (the block output
    # gradient, no-adapter towers)
    FUSE_Q8 = int(os.environ.get("LCCLIP_FP8_FUSE", "4"))
    # bf16 adapter towers: adapter + the following LayerNorm in one launch (LCCLIP_FUSE_LN=0: the
    # separate adapter_fwd + layernorm_fwd launches, for A/Bs)
    FUSE_LN = os.environ.get("LCCLIP_FUSE_LN", "1") != "0"

    def _fused_q8(self, level=1):
        return self.precision == "fp8" and self.FUSE_Q8 >= level

    def _gemm(self, st, name, A, epi, out0, **kw):
        """A [M, K] bf16 @ (staged weight `name`)^T: the bf16 GEMM, or in fp8 mode for the QKV /
        c_fc / c_proj weights the fp8 GEMM on A quantised here."""
        if self.precision == "fp8" and name in self.FP8_WEIGHTS:
            return ops.gemm_nt_fp8(ops.quant_fp8(A), st.q[name], epi, out0, **kw)
        return ops.gemm_nt(A, getattr(st, name), epi, out0, **kw)

    def _stage_lora(self, st, name, A, B, merges):
        """(A_pad [64,K], Bt_pad [64,N]) bf16 with rows >= r zero, staged from A [r,K], B [N,r]
        by two casts appended to `merges` (launched with the block's weight merges). The
        padding rows are zeroed once at allocation and never written (the casts cover rows < r
        only); the rank-r gradient kernels rely on that (ops.lora_grad_1p)."""
        r, K = A.shape
        N = B.shape[0]
        old = getattr(st, name, None)
        dev = A.device
        if old is None or old[0].shape[1] != K or old[1].shape[1] != N or old[0].dtype != self.dt:
            old = (torch.zeros((64, K), dtype=self.dt, device=dev),
                   torch.zeros((64, N), dtype=self.dt, device=dev),
                   _empty((N, r), self.dt, dev))
        a_pad, bt_pad, scratch = old
        merges.append((A.detach(), None, None, 0.0, a_pad[:r], None))
        merges.append((B.detach(), None, None, 0.0, scratch, bt_pad[:r]))
        return old

    # ------------------------------------------------------------------ forward
    def forward(self, x, n_seq: int, L: int, save: bool, training: bool = False, prompts=None,
                stop=None, replace=None, first_ln1=None, last_ln=None):
        """x: f32 [n_seq*L, D] residual stream, or float16 (the reference's autocast residual
        dtype, model.py:194-200 / 439-442: the fused adapter tower with last_ln, the LoRA tower,
        the frozen prompt towers of MVP / MaPLe). Returns (x_out, saved-per-layer or None).

        prompts: optional {layer: f32 [n_seq, P, D]} — prompt tokens appended to every sequence
        before that layer and dropped after it (prompt tuning, models/mvp_clip.py:158-175: cat
        along the sequence, block, x[:N]); that layer runs at L + P. Consecutive prompt layers
        with one prompt count keep the rows between them and overwrite them (the same values
        without the compact / expand copies). stop: run layers [0, stop)
        only (the MVP query pass, models/mvp_clip.py:211-216). replace: optional
        {layer: (row, f32 [P, D] or [n_seq, P, D])} — rows [row, row + P) of every sequence are
        overwritten before that layer (MaPLe's deep compound prompts,
        models/maple_clip/model.py:352-395). first_ln1: (y bf16 [M, D], mean, rstd) — the first
        block's ln_1 of x already computed (ops.vit_embed_ln), used when that block runs on x
        unchanged (no prompt rows appended or replaced there, bf16 operands). last_ln: {w, b, y,
        mean, rstd} — the LayerNorm after the stack (ln_post) fused into the last block's
        adapter (ops.adapter_ln_fwd): y bf16 [M, D] and its statistics over every row."""
        self.stage()
        M, D = x.shape
        xdt = x.dtype  # the residual stream's
        H = self.n_head
        dev = x.device
        P_of = {int(i): int(t.shape[1]) for i, t in (prompts or {}).items()}
        Mmax = n_seq * (L + max(P_of.values(), default=0))
        tmp_h = _empty((Mmax, D), self.dt, dev)
        q_g = ops.Fp8Mat(Mmax, 4 * D, dev) if self._fused_q8() else None
        q_h = ops.Fp8Mat(Mmax, D, dev) if self._fused_q8(2) else None  # ln_1 / ln_2 out, fp8
        tmp_g = _empty((Mmax, 4 * D), self.dt, dev) if q_g is None else None
        tmp_pre = None if save else _empty((Mmax, 4 * D), self.dt, dev)
        saved = [] if save else None
        # bf16 adapter towers: each adapter runs fused with the LayerNorm that reads its output
        # (ops.adapter_ln_fwd: ln_2 of the block, ln_1 of the next one); ln1_ready carries the
        # statistics of an ln_1 the previous block already wrote into tmp_h
        fuse_ln = (self.variant == "adapter" and q_h is None and D in (512, 768) and self.FUSE_LN)
        if xdt != F32 and not (self.variant == "vanilla" or (
                q_g is None and q_h is None and not prompts and not replace and stop is None
                and ((fuse_ln and last_ln is not None) or self.variant == "lora"))):
            raise ValueError("a half residual stream runs the fused adapter tower (with its "
                             "closing LayerNorm fused: last_ln) or the LoRA tower, bf16, without "
                             "prompt rows, or the frozen (prompt) tower")
        e_resid = EPI_RESID16 if xdt == F16 else EPI_RESID
        ln1_ready = None
        n_run = len(self.blocks) if stop is None else min(stop, len(self.blocks))
        carried = 0  # prompt rows x carries from the previous layer (kept: same count here)
        for idx, (blk, st) in enumerate(zip(self.blocks, self.staged)):
            if stop is not None and idx >= stop:
                break
            if replace and idx in replace:
                r0, pr = replace[idx]
                if idx == 0:
                    x = x.clone()  # never write into the caller's input
                x.view(n_seq, -1, D)[:, r0:r0 + pr.shape[-2]] = pr
            P = P_of.get(idx, 0)
            Lx = L + P
            Mx = n_seq * Lx
            inherit = bool(P) and carried == P
            if inherit:
                # the previous layer's prompt rows are dropped and this layer's appended in their
                # place (models/mvp_clip.py:163-175: x[:N] then cat): overwrite them in x, which
                # no saved tensor aliases (the previous layer saved its input, not its output)
                x.view(n_seq, Lx, D)[:, L:] = prompts[idx]
            elif P:
                xe = _empty((Mx, D), xdt, dev)  # prompt rows cast to the stream's dtype
                v = xe.view(n_seq, Lx, D)
                v[:, :L] = x.view(n_seq, L, D)
                v[:, L:] = prompts[idx]
                x = xe
            th = tmp_h[:Mx]
            s = {}
            mean1 = _empty((Mx,), F32, dev)
            rstd1 = _empty((Mx,), F32, dev)
            h1 = _empty((Mx, D), self.dt, dev) if (save and self.variant == "lora") else th
            qkv = _empty((Mx, 3 * D), self.dt, dev)
            if q_h is not None:  # bf16 h1 only when LoRA's gradient reads it
                qa = ops.layernorm_fwd_fp8(x, blk.ln_1.weight, blk.ln_1.bias, q_h.narrow(Mx),
                                           mean1, rstd1, y=None if h1 is th else h1)
                ops.gemm_nt_fp8(qa, st.q["wqkv"], EPI_BF16, qkv, bias=blk.attn.in_proj_bias)
            else:
                if ln1_ready is not None:  # written by the previous block's fused adapter
                    mean1, rstd1 = ln1_ready
                elif (idx == 0 and first_ln1 is not None and P == 0
                      and not (replace and 0 in replace)):
                    h1, mean1, rstd1 = first_ln1
                else:
                    ops.layernorm_fwd(x, blk.ln_1.weight, blk.ln_1.bias, h1, mean1, rstd1)
                self._gemm(st, "wqkv", h1, EPI_BF16, qkv, bias=blk.attn.in_proj_bias)
            ln1_ready = None
            O = _empty((Mx, D), self.dt, dev)
            lse = _empty((n_seq * H, Lx), F32, dev)
            ops.attn_fwd(qkv, O, lse, n_seq, Lx, H, self.causal)
            x_mid = _empty((Mx, D), xdt, dev)
            if self.variant == "adapter":
                ad = blk.adaptmlp
                keep = 1.0 - ad.dropout if (training and ad.dropout > 0) else 1.0
                seed1 = next(_seed_counter) * 0x9E3779B1
                z1 = _empty((Mx, D), self.dt, dev)
                ops.gemm_nt(O, st.wo, EPI_BF16, z1, bias=blk.attn.out_proj.bias)
                hd1 = _empty((Mx, ad.down_size), self.dt, dev)
                mean2 = _empty((Mx,), F32, dev)
                rstd2 = _empty((Mx,), F32, dev)
                if fuse_ln and q_g is None:
                    ops.adapter_ln_fwd(z1, st.wd, ad.down_proj.bias, st.wu, ad.up_proj.bias,
                                       ad.scale, keep, seed1, x, x_mid, hd1, blk.ln_2.weight,
                                       blk.ln_2.bias, th, mean2, rstd2, seed_dev=self.seed_dev)
                    ln2_done = True
                else:
                    ops.adapter_fwd(z1, st.wd, ad.down_proj.bias, st.wu, ad.up_proj.bias, ad.scale,
                                    keep, seed1, x, x_mid, hd1, seed_dev=self.seed_dev)
                    ln2_done = False
                s.update(z1=z1, hd1=hd1, keep=keep)
            else:
                ops.gemm_nt(O, st.wo, e_resid, x_mid, bias=blk.attn.out_proj.bias, aux=x)
                mean2 = _empty((Mx,), F32, dev)
                rstd2 = _empty((Mx,), F32, dev)
                ln2_done = False
            pre = _empty((Mx, 4 * D), self.dt, dev) if save else tmp_pre[:Mx]
            # training saves QuickGELU'(pre) (the c_fc dX epilogue is then a plain multiply)
            if q_g is not None:
                # ln_2 and QuickGELU(pre) only as the fp8 operands of c_fc / c_proj (inference
                # discards QuickGELU')
                if q_h is not None:
                    qa = ops.layernorm_fwd_fp8(x_mid, blk.ln_2.weight, blk.ln_2.bias,
                                               q_h.narrow(Mx), mean2, rstd2)
                else:
                    ops.layernorm_fwd(x_mid, blk.ln_2.weight, blk.ln_2.bias, th, mean2, rstd2)
                    qa = ops.quant_fp8(th)
                g_in = ops.gemm_nt_fp8(qa, st.q["wfc"], EPI_GELU_D_Q8, pre,
                                       bias=blk.mlp.c_fc.bias, q_out=q_g.narrow(Mx))
                wpr = lambda epi, out0, **kw: ops.gemm_nt_fp8(g_in, st.q["wpr"], epi, out0, **kw)  # noqa: E731
            else:
                if not ln2_done:
                    ops.layernorm_fwd(x_mid, blk.ln_2.weight, blk.ln_2.bias, th, mean2, rstd2)
                self._gemm(st, "wfc", th, EPI_GELU_D if save else EPI_GELU, pre,
                           bias=blk.mlp.c_fc.bias, out1=tmp_g[:Mx])
                wpr = lambda epi, out0, **kw: self._gemm(st, "wpr", tmp_g[:Mx], epi, out0, **kw)  # noqa: E731
            x_out = _empty((Mx, D), xdt, dev)
            if self.variant == "adapter":
                ad = blk.adaptmlp
                seed2 = next(_seed_counter) * 0x9E3779B1
                z2 = _empty((Mx, D), self.dt, dev)
                wpr(EPI_BF16, z2, bias=blk.mlp.c_proj.bias)
                hd2 = _empty((Mx, ad.down_size), self.dt, dev)
                nxt = idx + 1
                if (fuse_ln and nxt < len(self.blocks) and (stop is None or nxt < stop)
                        and not P_of.get(nxt, 0) and not P and not (replace and nxt in replace)):
                    # the next block's ln_1 into tmp_h (c_fc has consumed it by now: same stream)
                    nb = self.blocks[nxt]
                    m1 = _empty((Mx,), F32, dev)
                    r1 = _empty((Mx,), F32, dev)
                    ops.adapter_ln_fwd(z2, st.wd, ad.down_proj.bias, st.wu, ad.up_proj.bias,
                                       ad.scale, s["keep"], seed2, x_mid, x_out, hd2,
                                       nb.ln_1.weight, nb.ln_1.bias, th, m1, r1,
                                       seed_dev=self.seed_dev)
                    ln1_ready = (m1, r1)
                elif (last_ln is not None and fuse_ln and nxt == len(self.blocks) and not P
                      and stop is None):
                    # the LayerNorm after the stack (ln_post) over every row
                    ops.adapter_ln_fwd(z2, st.wd, ad.down_proj.bias, st.wu, ad.up_proj.bias,
                                       ad.scale, s["keep"], seed2, x_mid, x_out, hd2,
                                       last_ln["w"], last_ln["b"], last_ln["y"], last_ln["mean"],
                                       last_ln["rstd"], seed_dev=self.seed_dev)
                    last_ln["done"] = True
                else:
                    ops.adapter_fwd(z2, st.wd, ad.down_proj.bias, st.wu, ad.up_proj.bias, ad.scale,
                                    s["keep"], seed2, x_mid, x_out, hd2, seed_dev=self.seed_dev)
                s.update(z2=z2, hd2=hd2)
            else:
                wpr(e_resid, x_out, bias=blk.mlp.c_proj.bias, aux=x_mid)
            # a run of prompt layers with one prompt count keeps the rows between them (no
            # compact-and-expand copies): the next layer overwrites them
            pkeep = (self.PROMPT_KEEP and bool(P) and idx + 1 < n_run
                     and P_of.get(idx + 1, 0) == P and not (replace and idx + 1 in replace))
            if save:
                s.update(x_in=x, mean1=mean1, rstd1=rstd1, qkv=qkv, O=O, lse=lse, x_mid=x_mid,
                         mean2=mean2, rstd2=rstd2, gd=pre, P=P, pkeep=pkeep, inherit=inherit)
                if replace and idx in replace:
                    s["R"] = (replace[idx][0], replace[idx][1].shape[-2])
                if self.variant == "lora":
                    s["h1"] = h1
                saved.append(s)
            if not P or pkeep:
                x, carried = x_out, (P if pkeep else 0)
            else:
                x, carried = x_out.view(n_seq, Lx, D)[:, :L].reshape(n_seq * L, D), 0
        return x, saved

    # ------------------------------------------------------------------ backward
    def backward(self, saved, dx, dxb, grads, n_seq: int, L: int, on_layer=None,
                 grad_stream=None, need_dx: bool = True, prompt_grads=None,
                 keep_input: bool = False, gscale=None):
        """dx f32 / dxb bf16 [rows, D]: gradient w.r.t. the stack output. grads: dict
        param -> f32 tensor (accumulated). on_layer(li) is called once layer li's PEFT gradients
        have been launched (layers run last to first). Returns (dx, dxb) w.r.t. the stack input.

        grad_stream: optional side HIP stream for the PEFT weight-gradient reductions (adapter
        dW/db, LoRA dA/dB), which feed only `grads`: they run beside the dX chain's MFMA-bound
        GEMMs. Each layer waits for the previous layer's side work before rewriting the shared
        gradient buffers the side reads; sync_grads() joins it (done before returning).

        need_dx=False (a tower whose input is frozen: patch / token embeddings): nothing below
        layer 0's first trainable parameter needs a gradient, so its out-proj dX, attention
        backward, QKV dX and ln_1 backward are skipped, as the reference's autograd skips them
        (adapter: all of them, dz included; LoRA: the attention backward stays for the in-proj
        LoRA gradients). Returns (None, None) then.

        prompt_grads: dict filled with {layer: f32 [n_seq, P, D]}, the gradient w.r.t. the
        prompt tokens the forward appended at that layer (their rows of the layer's input
        gradient; the dropped rows of its output carry zero gradient), and {('R', layer):
        f32 [n_seq, P, D]} for the rows the forward replaced there (those rows' input gradient,
        which then stops: zeroed below that layer).

        keep_input: never write into (dx, dxb) (a caller-kept buffer, ImageTower._grad_in); the
        layers' output gradients then ping-pong between two other pairs.

        dx float16 (the half residual stream's gradient, the fused adapter tower): every residual
        gradient is stored in half, carrying the power-of-two scale `gscale` (device f32 [1],
        set by the caller: ops.grad_pow2_normalize) that the weight gradients divide out. The
        adapter tower then keeps no bf16 copies (dxb may be None): its adapter backward and
        weight-gradient launches read the half gradient directly (ops.adapter_bwd / _wgrad
        _g16 forms, bit-identical to reading the copy)."""
        M, D = dx.shape
        gdt = dx.dtype
        if gdt != F32 and (gscale is None or prompt_grads is not None
                           or any(s.get("P", 0) or "R" in s for s in saved)):
            raise ValueError("a half residual gradient needs its gscale and no prompt rows")
        self._gscale = gscale
        # the half gradient's consumers read it directly: no bf16 copies (LayerNorm backward
        # writes the half gradient only)
        nocopy = gdt != F32 and self.half_grad_direct()
        cdt = None if nocopy else self.dt  # the copies' type (None: not kept)
        main = torch.cuda.current_stream(dx.device)
        self._gs = grad_stream
        ev = None
        H = self.n_head
        dev = dx.device
        Mmax = n_seq * (L + max((s.get("P", 0) for s in saved), default=0))
        q_da = ops.Fp8Mat(Mmax, 4 * D, dev) if self._fused_q8() else None
        # the attention backward's dq|dk|dv as the fp8 QKV dX operand (LoRA reads them in bf16)
        fuse_attn = self._fused_q8(3) and self.variant != "lora" and Mmax // n_seq <= 224
        q_dqkv = ops.Fp8Mat(Mmax, 3 * D, dev) if fuse_attn else None
        da = _empty((Mmax, 4 * D), self.dt, dev) if q_da is None else None
        dh = _empty((Mmax, D), self.dt, dev)
        dO = _empty((Mmax, D), self.dt, dev)
        dqkv = _empty((Mmax, 3 * D), self.dt, dev)
        dz = _empty((Mmax, D), self.dt, dev) if self.variant == "adapter" else None
        dx_mid = _empty((Mmax, D), gdt, dev)
        dx_midb = _empty((Mmax, D), cdt, dev)
        # output-gradient buffers: the incoming pair and one more (ping-pong); prompt layers
        # expand the current gradient into a free pair and compact their output back
        pairs = [(dx, None if nocopy else dxb),
                 (_empty((Mmax, D), gdt, dev), _empty((Mmax, D), cdt, dev))]
        if keep_input:
            pairs.append((_empty((Mmax, D), gdt, dev), _empty((Mmax, D), cdt, dev)))
        cur = 0
        # fp8 (no adapter: the block output gradient feeds c_proj dX directly): ln_1's backward
        # also writes its result as the fp8 operand of the next (lower) block's c_proj dX GEMM
        # (ops.layernorm_bwd_fp8), so that block skips quant_fp8. q_of[i]: the fp8 image of
        # pairs[i]'s bf16 gradient while it is current (dropped when prompt rows change it).
        fuse_ln_q = self._fused_q8(4) and self.variant != "adapter" and D % 256 == 0
        q_mats, q_of = {}, {}
        for li in range(len(self.blocks) - 1, -1, -1):
            blk, st, s = self.blocks[li], self.staged[li], saved[li]
            if ev is not None:
                main.wait_event(ev)  # side reads of the buffers this layer rewrites are done
            P = s.get("P", 0)
            Lx = L + P
            Mx = n_seq * Lx
            if P and len(pairs) == 2:
                pairs.append((_empty((Mmax, D), F32, dev), _empty((Mmax, D), self.dt, dev)))
            if P and not s.get("pkeep"):  # (kept rows: the gradient is already in the Lx layout)
                e = 2 if cur != 2 else 1
                q_of.clear()
                for src, dst in zip(pairs[cur], pairs[e]):
                    v = dst[:Mx].view(n_seq, Lx, D)
                    v[:, :L] = src[:M].view(n_seq, L, D)
                    v[:, L:] = 0
                cur = e
            gx, gxb = _rows(pairs[cur][0], Mx), _rows(pairs[cur][1], Mx)
            out = next(i for i in range(len(pairs)) if i != cur and (
                i != 0 or (not keep_input and (P == 0 or pairs[0][0].shape[0] >= Mx))))
            ox, oxb = _rows(pairs[out][0], Mx), _rows(pairs[out][1], Mx)
            # ---- MLP sub-block: x_out = x_mid + [A](c_proj(gelu(c_fc(ln_2(x_mid)))))
            if self.variant == "adapter":
                dY = self._adapter_bwd(blk, st, gx if nocopy else gxb, s["hd2"], s["z2"],
                                       s["keep"], dz[:Mx], grads)
            else:
                dY = gxb
            if q_da is not None:
                qdy = q_of.pop(cur, None) if self.variant != "adapter" else None
                qdy = qdy if qdy is not None and qdy.rows == Mx else ops.quant_fp8(dY)
                q = ops.gemm_nt_fp8(qdy, st.q["wprT"], EPI_MUL_Q8, None, aux=s["gd"],
                                    q_out=q_da.narrow(Mx))
                ops.gemm_nt_fp8(q, st.q["wfcT"], EPI_BF16, dh[:Mx])
            else:
                self._gemm(st, "wprT", dY, EPI_MUL, da[:Mx], aux=s["gd"])
                self._gemm(st, "wfcT", da[:Mx], EPI_BF16, dh[:Mx])
            ops.layernorm_bwd(dh[:Mx], s["x_mid"], s["mean2"], s["rstd2"], blk.ln_2.weight,
                              dx_mid[:Mx], _rows(dx_midb, Mx), dres=gx)
            # ---- attention sub-block: x_mid = x_in + [A](out_proj(attn(ln_1(x_in))))
            first = li == 0 and not need_dx
            if self.variant == "adapter":
                dY = self._adapter_bwd(blk, st, dx_mid[:Mx] if nocopy else dx_midb[:Mx],
                                       s["hd1"], s["z1"], s["keep"], None if first else dz[:Mx],
                                       grads)
            else:
                dY = dx_midb[:Mx]
            if first and self.variant != "lora":
                self._layer_done(li, grad_stream, on_layer)
                break
            ops.gemm_nt(dY, st.woT, EPI_BF16, dO[:Mx])
            attn = blk.attn
            if self.variant == "lora":
                self._lora_grad(dY, s["O"], attn.out_proj.lora_A, attn.out_proj.lora_B,
                                attn.scaling, grads, st.lora_out)
            if q_dqkv is not None and not first:
                qd = ops.attn_bwd_fp8(s["qkv"], s["O"], dO[:Mx], s["lse"], q_dqkv.narrow(Mx), n_seq,
                                      Lx, H, self.causal)
            else:
                qd = None
                ops.attn_bwd(s["qkv"], s["O"], dO[:Mx], s["lse"], dqkv[:Mx], n_seq, Lx, H,
                             self.causal)
            if self.variant == "lora":
                self._lora_grad(dqkv[:Mx], s["h1"], attn.in_proj_weight_lora_A,
                                attn.in_proj_weight_lora_B, attn.scaling, grads, st.lora_in)
            if first:
                self._layer_done(li, grad_stream, on_layer)
                break
            if qd is not None:
                ops.gemm_nt_fp8(qd, st.q["wqkvT"], EPI_BF16, dh[:Mx])
            else:
                self._gemm(st, "wqkvT", dqkv[:Mx], EPI_BF16, dh[:Mx])
            if fuse_ln_q and "R" not in s and not P:
                if out not in q_mats:
                    q_mats[out] = ops.Fp8Mat(Mmax, D, dev)
                q_of[out] = ops.layernorm_bwd_fp8(dh[:Mx], s["x_in"], s["mean1"], s["rstd1"],
                                                  blk.ln_1.weight, ox, oxb, q_mats[out].narrow(Mx),
                                                  dres=dx_mid[:Mx])
            else:
                q_of.pop(out, None)
                ops.layernorm_bwd(dh[:Mx], s["x_in"], s["mean1"], s["rstd1"], blk.ln_1.weight, ox,
                                  oxb, dres=dx_mid[:Mx])
            ev = self._layer_done(li, grad_stream, on_layer)
            if "R" in s:
                r0, pr = s["R"]
                if prompt_grads is not None:
                    prompt_grads[("R", li)] = ox.view(n_seq, Lx, D)[:, r0:r0 + pr].clone()
                ox.view(n_seq, Lx, D)[:, r0:r0 + pr] = 0
                oxb.view(n_seq, Lx, D)[:, r0:r0 + pr] = 0
            if P:
                if ev is not None:
                    main.wait_event(ev)  # the side stream read the expanded gradient
                v = ox.view(n_seq, Lx, D)
                if prompt_grads is not None:
                    prompt_grads[li] = v[:, L:].clone()
                if s.get("inherit"):
                    # these prompt rows replaced the previous layer's (dropped) ones: no gradient
                    # flows into them; the layout stays Lx for the previous layer
                    v[:, L:] = 0
                    oxb.view(n_seq, Lx, D)[:, L:] = 0
                    cur = out
                else:
                    # compact into the (consumed) expanded pair
                    pairs[cur][0][:M].view(n_seq, L, D).copy_(v[:, :L])
                    pairs[cur][1][:M].view(n_seq, L, D).copy_(oxb.view(n_seq, Lx, D)[:, :L])
            else:
                cur = out
        self.sync_grads()
        self._gscale = None
        if not need_dx:
            return None, None
        return pairs[cur][0][:M], _rows(pairs[cur][1], M)

    @staticmethod
    def _layer_done(li, grad_stream, on_layer):
        ev = None
        if grad_stream is not None:
            ev = torch.cuda.Event()
            ev.record(grad_stream)
        if on_layer is not None:
            on_layer(li)
        return ev

    def sync_grads(self):
        """Make the current stream wait for the PEFT-gradient work on the side stream."""
        gs = getattr(self, "_gs", None)
        if gs is not None:
            torch.cuda.current_stream(gs.device).wait_stream(gs)

    def _side(self):
        """Context for launching gradient reductions: the side stream (after the work that
        produced their inputs on the current stream) or the current stream."""
        gs = getattr(self, "_gs", None)
        if gs is None:
            return _Null()
        gs.wait_stream(torch.cuda.current_stream(gs.device))
        return torch.cuda.stream(gs)

    @staticmethod
    def _grad(grads, p):
        g = grads.get(p)
        if g is None:
            raise KeyError("missing gradient buffer for a trainable parameter")
        return g

    def _adapter_bwd(self, blk, st, gout, h, z, keep, dz, grads):
        ad = blk.adaptmlp
        M = gout.shape[0]
        dpre = _empty((M, ad.down_size), self.dt, gout.device)
        ops.adapter_bwd(gout, h, st.wuT, st.wdT, ad.scale, keep, dpre, dz)  # dz None: dpre only
        with self._side():
            if getattr(self, "_gs", None) is not None:
                dpre.record_stream(self._gs)
            ops.adapter_wgrad(gout, h, z, dpre, ad.scale, self._grad(grads, ad.up_proj.weight),
                              self._grad(grads, ad.up_proj.bias),
                              self._grad(grads, ad.down_proj.weight),
                              self._grad(grads, ad.down_proj.bias),
                              gscale=getattr(self, "_gscale", None))
        return dz

    # LCCLIP_HALF_GRAD_DIRECT=0: the adapter tower's half residual gradient with bf16 copies for
    # its adapter backward launches, as before lc_adapter_*_g16 (A/B experiments)
    HALF_GRAD_DIRECT = os.environ.get("LCCLIP_HALF_GRAD_DIRECT", "1") != "0"

    def half_grad_direct(self):
        """A half residual gradient's consumers read it directly (no bf16 copies): the adapter
        tower (its adapter backward launches have _g16 forms)."""
        return self.variant == "adapter" and self.HALF_GRAD_DIRECT

    # LCCLIP_PROMPT_KEEP=0: compact and re-expand between prompt layers of one prompt count
    # (A/B experiments)
    PROMPT_KEEP = os.environ.get("LCCLIP_PROMPT_KEEP", "1") != "0"
    # LCCLIP_MERGE_BATCH=0: one lc_merge_weight launch per LoRA merge / cast (A/B experiments)
    MERGE_BATCH = os.environ.get("LCCLIP_MERGE_BATCH", "1") != "0"
    # LCCLIP_LORA_1P=0: the four-GEMM form (A/B experiments)
    LORA_1P = os.environ.get("LCCLIP_LORA_1P", "1") != "0"

    def _lora_1p(self, r, K, N):
        return self.LORA_1P and r <= 4 and (K, N) in ((768, 2304), (768, 768), (512, 1536),
                                                      (512, 512))

    def lora_half_grad_ok(self):
        """Every LoRA gradient of this (LoRA) stack runs ops.lora_grad_1p, the form that divides
        out the half residual gradient's scale."""
        for blk in self.blocks:
            a = blk.attn
            for A, B in ((a.in_proj_weight_lora_A, a.in_proj_weight_lora_B),
                         (a.out_proj.lora_A, a.out_proj.lora_B)):
                if not self._lora_1p(A.shape[0], A.shape[1], B.shape[0]):
                    return False
        return True

    def _lora_grad(self, dY, X, A, B, scaling, grads, padded):
        """Rank-r LoRA gradients (lora.py:838-839, 1073-1074 autograd): one pass over X and dY
        (ops.lora_grad_1p: XA = X A^T and dYB = dY B per 32-row block, dB += s dY^T XA and
        dA += s dYB^T X from the same staged rows), or for shapes it does not cover four
        streaming GEMMs: XA and dYB (skinny, [M,64] bf16 with zero columns >= r), then
        dB += s dY^T XA and dA += s dYB^T X (gemm_tn, outputs masked to r)."""
        a_pad, bt_pad, _ = padded
        M = dY.shape[0]
        r, K = A.shape
        N = B.shape[0]
        gsc = getattr(self, "_gscale", None)  # dY carries the half residual gradient's scale
        if self._lora_1p(r, K, N):
            with self._side():
                ops.lora_grad_1p(dY, X, a_pad, bt_pad, r, scaling, self._grad(grads, A),
                                 self._grad(grads, B), gscale=gsc)
            return
        if gsc is not None:
            raise ValueError("a scaled LoRA gradient runs the one-pass kernel only")
        with self._side():
            xa = _empty((M, 64), self.dt, dY.device)
            dyb = _empty((M, 64), self.dt, dY.device)
            gs = getattr(self, "_gs", None)
            if gs is not None:
                xa.record_stream(gs)
                dyb.record_stream(gs)
            ops.gemm_nt(X, a_pad, EPI_BF16, xa)
            ops.gemm_nt(dY, bt_pad, EPI_BF16, dyb)
            ops.gemm_tn(dY, xa, self._grad(grads, B), alpha=scaling)
            ops.gemm_tn(dyb, X, self._grad(grads, A), alpha=scaling)


class ScaledGrads:
    """A backward run on a power-of-two-scaled incoming gradient (IEEE-half storage: its 16-bit
    gradient copies sit mostly below half's normal range at ViT-B/16, 1e-9..3e-4). The scale is
    computed on the device (ops.grad_pow2_normalize: the role of the reference's GradScaler,
    methods/adapter_clip.py:93); the stack's PEFT gradients accumulate in a zeroed scratch
    buffer and are added to the caller's divided by that scale, and so are any f32 input /
    prompt gradients (exact: a power of two, no host sync, no skipped steps)."""

    def __init__(self, stack, df, target_exp=10):
        dev = df.device
        self.stack = stack
        self.df = df.contiguous().float().clone()
        self.scale = _empty((1,), F32, dev)
        ops.grad_pow2_normalize(self.df, self.scale, target_exp=target_exp)
        params = stack.trainable_params()
        self.flat = torch.zeros(sum(p.numel() for p in params), dtype=F32, device=dev)
        self.grads, off = {}, 0
        for p in params:
            self.grads[p] = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def add_to(self, dst):
        """dst[p] += scratch[p] / scale: one launch when dst's buffers are consecutive views of
        one flat buffer in parameter order (the trainer's flat gradient), else one per
        parameter."""
        params = self.stack.trainable_params()
        if not params:
            return
        views = [dst[p] for p in params]
        first = views[0]
        contiguous = True
        off = 0
        for v in views:
            if not v.is_contiguous() or v.data_ptr() != first.data_ptr() + off * 4:
                contiguous = False
                break
            off += v.numel()
        if contiguous:
            span = torch.as_strided(first, (self.flat.numel(),), (1,))
            ops.add_unscaled(span, self.flat, self.scale)
            return
        for p in params:
            ops.add_unscaled(dst[p], self.grads[p], self.scale)

    def unscaled(self, t):
        """A fresh f32 tensor t / scale."""
        if t is None:
            return None
        out = torch.zeros(t.shape, dtype=F32, device=t.device)
        ops.add_unscaled(out.view(-1), t.contiguous().view(-1), self.scale)
        return out


class RowGrad:
    """The stack-output gradient pair (f32, bf16 [rows, D]) of a tower whose head reads a few
    rows per sequence: the row-gathered LayerNorm backward (ln_post at the CLS rows,
    model.py:782; ln_final at the EOT rows, model.py:954) writes those rows and every other row
    is zero. One pair is kept across steps (BlockStack.backward(keep_input=True) never writes
    it) instead of a per-step full-buffer fill (232 MB at B = 256): before each use the rows the
    previous use wrote are zeroed again, unless `key` says they are the same rows (the image
    tower's CLS rows are fixed by (n, L)). A larger shape reallocates; a smaller one uses a
    prefix whose other rows are zero by the same invariant."""

    def __init__(self):
        self.buf = None
        self.prev = None       # int64 rows written by the previous use
        self.prev_key = None

    def get(self, rows, D, dev, idx, key=None, dt=BF16, gdt=F32):
        """dt: the 16-bit copy's type; gdt: the gradient's (f32, or float16 for the half
        residual stream)."""
        b = self.buf
        if dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
            # graph-pool memory: fresh zeros, captured as part of the graph, not kept
            return (torch.zeros((rows, D), dtype=gdt, device=dev),
                    torch.zeros((rows, D), dtype=dt, device=dev))
        if (b is None or b[0].shape[0] < rows or b[0].shape[1] != D or b[0].device != dev
                or b[1].dtype != dt or b[0].dtype != gdt):
            self.buf = b = (torch.zeros((rows, D), dtype=gdt, device=dev),
                            torch.zeros((rows, D), dtype=dt, device=dev))
        elif self.prev is not None and (key is None or key != self.prev_key):
            for t in b:
                t.index_fill_(0, self.prev, 0)
        self.prev, self.prev_key = idx.to(torch.int64), key
        return b[0][:rows], b[1][:rows]


class ImageTower:
    """VisualTransformer.forward (model.py:755-787) on the engine."""

    def __init__(self, visual, stack: BlockStack):
        self.visual = visual
        self.stack = stack
        self._key = None
        self._grad_in = RowGrad()  # ln_post's backward writes the CLS rows only
        self._gsc = None  # the half residual gradient's scale (device f32 [1])

    def _stage(self):
        v = self.visual
        dt = self.stack.dt
        key = _key(v.conv1.weight, v.proj) + (dt,)
        if key != self._key:
            W = v.conv1.weight.shape[0]
            dev = v.conv1.weight.device
            self.conv_w = _empty((W, v.conv1.weight[0].numel()), dt, dev)
            ops.merge_weight(v.conv1.weight.detach().reshape(W, -1), None, None, 0.0, self.conv_w)
            E = v.proj.shape[1]
            self.projT = _empty((E, W), dt, dev)      # forward: f = x @ proj  -> B = proj^T
            self.proj = _empty((W, E), dt, dev)       # backward: dx = df @ proj^T -> B = proj
            ops.merge_weight(v.proj.detach(), None, None, 0.0, self.proj, self.projT)
            self._key = key

    def embed(self, img, extra=None, keep=None):
        """conv1 + CLS/pos + ln_pre (model.py:756-766): (x0 f32 [n*L, D], n, L); x0 float16
        for the half residual stream (_resid16).
        extra: optional f32 [P, D] rows appended to every sequence after the positional
        embedding and before ln_pre (MaPLe's shared visual context,
        models/maple_clip/model.py:566-575); L then counts them. keep: dict that receives what
        embed_backward() needs."""
        pe, n, npch = self._patch_embed(img)
        x0, n, L = self._embed_tail(pe, n, npch, extra, keep)
        if self.stack.variant == "vanilla" and self._resid16():  # the frozen prompt towers
            x0 = x0.half()
        return x0, n, L

    def _patch_embed(self, img):
        """conv1 as a GEMM on im2col rows: (f32 [n*np, D], n, np)."""
        v = self.visual
        self._stage()
        dev = img.device
        P = v.patch_size
        g = v.input_resolution // P
        npch = g * g
        if img.dim() == 2:
            # conv1's bf16 im2col rows, already produced by the fused train transform
            # (lcclip.transforms.TrainTransform(..., layout="patches"))
            if img.dtype != BF16 or img.shape[1] != 3 * P * P or img.shape[0] % npch:
                raise ValueError(f"patch input must be bf16 [n*{npch}, {3 * P * P}]")
            n = img.shape[0] // npch
            # (the fp16 tower: bf16 -> half is exact for normalised pixels, |x| < 2^15)
            patches = img.contiguous().to(self.stack.dt)
        else:
            n = img.shape[0]
            img = img.contiguous().to(F32)
            patches = _empty((n * npch, 3 * P * P), self.stack.dt, dev)
            ops.patchify(img, P, patches)
        pe = _empty((n * npch, v.width), F32, dev)
        ops.gemm_nt(patches, self.conv_w, EPI_F32, pe)
        return pe, n, npch

    def _embed_tail(self, pe, n, npch, extra, keep):
        v = self.visual
        dev = pe.device
        L, D = npch + 1, v.width
        xa = _empty((n * L, D), F32, dev)
        ops.vit_assemble(pe, v.class_embedding, v.positional_embedding, xa, n, npch)
        if extra is not None:
            P = extra.shape[0]
            xe = _empty((n * (L + P), D), F32, dev)
            ve = xe.view(n, L + P, D)
            ve[:, :L] = xa.view(n, L, D)
            ve[:, L:] = extra.detach().float()
            xa, L = xe, L + P
        x0 = _empty((n * L, D), F32, dev)
        mean = rstd = None
        if keep is not None:
            mean = _empty((n * L,), F32, dev)
            rstd = _empty((n * L,), F32, dev)
            keep.update(xa=xa, mean=mean, rstd=rstd, n=n, L=L)
        ops.layernorm_fwd(xa, v.ln_pre.weight, v.ln_pre.bias, x0, mean, rstd)
        return x0, n, L

    def embed_backward(self, keep, dx0, rows):
        """Gradient w.r.t. the rows [rows, L) embed(extra=...) appended, summed over the
        sequences: ln_pre backward of the input gradient dx0 f32 [n*L, D] (the rest of the
        embedding is frozen)."""
        v = self.visual
        n, L = keep["n"], keep["L"]
        D = v.width
        dxa = _empty((n * L, D), F32, dx0.device)
        ops.layernorm_bwd(dx0, keep["xa"], keep["mean"], keep["rstd"], v.ln_pre.weight, dxa, None)
        return dxa.view(n, L, D)[:, rows:].sum(0)

    def _ln_post(self, x, n, L, out_dtype):
        v = self.visual
        dev = x.device
        cls_idx = torch.arange(n, device=dev, dtype=torch.int32) * L
        lnp = _empty((n, v.width), out_dtype, dev)
        mean = _empty((n,), F32, dev)
        rstd = _empty((n,), F32, dev)
        ops.layernorm_fwd(x, v.ln_post.weight, v.ln_post.bias, lnp, mean, rstd, row_idx=cls_idx)
        return lnp, cls_idx, mean, rstd

    def query(self, x0, n, L, stop=None, first_ln1=None):
        """The MVP key query (models/mvp_clip.py:196-218): blocks [0, stop) on x0 without
        saving, then ln_post of the CLS rows (f32 [n, D], no projection). first_ln1: layer 0's
        ln_1 of x0 from embed_query()."""
        x, _ = self.stack.forward(x0, n, L, save=False, stop=stop, first_ln1=first_ln1)
        return self._ln_post(x, n, L, F32)[0]

    def embed_query(self, img):
        """embed() for the MVP passes, (x0, n, L, first_ln1 or None): the half residual stream's
        fused embed (conv1 rows -> CLS / pos -> ln_pre -> x0 in half, and layer 0's ln_1 for the
        key query, which runs on x0 unchanged) where it applies, else embed()."""
        if (self.FUSE_EMBED and self._resid16() and self.stack.variant == "vanilla"
                and self.stack.precision == "bf16"):
            return self.embed_ln1(img, half=True)
        x0, n, L = self.embed(img)
        return x0, n, L, None

    def forward(self, img, save: bool, training: bool = False, prompts=None):
        """img -> (features f32 [n, E], ctx). prompts: {layer: f32 [n, P, D]} appended before
        that layer (prompt tuning, models/mvp_clip.py:158-175)."""
        if (self.FUSE_EMBED and not prompts and self.stack.precision == "bf16"
                and self.visual.width in (512, 768, 1024)):
            x0, n, L, first = self.embed_ln1(img, half=self._resid16())
            return self.forward_embedded(x0, n, L, save, training, prompts, first_ln1=first)
        x0, n, L = self.embed(img)
        return self.forward_embedded(x0, n, L, save, training, prompts)

    # the patch embedding's CLS / positional add, ln_pre and the first ln_1 in one launch
    # (False: the three separate launches, for A/Bs)
    FUSE_EMBED = True
    # the residual stream in IEEE half, the reference's autocast dtype (model.py:194-200: its
    # LayerNorm returns the input dtype, so x is fp16 from conv1 through every block; the fused
    # adapter, LoRA and frozen prompt towers: lc_*_x16, LC_EPI_RESID16): a third less HBM traffic
    # in the residual adds, the fused adapter + LayerNorm forward and the x read of every
    # LayerNorm backward. False: the f32 stream (A/Bs)
    RESID16 = True
    GRAD_EXP = 12  # the half residual gradient's scale target, 2^GRAD_EXP <= max|dL/df| s < 2^13
    # LCCLIP_HALF_GRAD=0: a half residual stream with an f32 gradient (A/B experiments)
    HALF_GRAD = os.environ.get("LCCLIP_HALF_GRAD", "1") != "0"

    def _resid16(self):
        st = self.stack
        if not (self.RESID16 and self.visual.width in (512, 768)) or st.dt != BF16:
            # (the fp16 tower, image_precision="fp16": an f32 residual stream, its 16-bit
            # operands in IEEE half)
            return False
        if st.variant == "vanilla":
            # the frozen prompt towers (MVP, MaPLe; bf16 or fp8 GEMMs): the reference casts
            # their prompt rows to the stream's dtype (mvp_clip.py:256-257, maple.py:243);
            # the residual gradient stays f32 (the prompt gradients are read from its rows)
            return True
        return (self.FUSE_EMBED and st.precision == "bf16"
                and ((st.variant == "adapter" and st.FUSE_LN) or st.variant == "lora"))

    def embed_ln1(self, img, half=False):
        """embed() and the first block's ln_1 in one launch (ops.vit_embed_ln): (x0, n, L,
        (ln_1(x0) bf16, mean1, rstd1)) for BlockStack.forward(first_ln1=...). half: x0 in IEEE
        half (the half residual stream)."""
        v = self.visual
        pe, n, npch = self._patch_embed(img)
        L, D = npch + 1, v.width
        dev = pe.device
        x0 = _empty((n * L, D), F16 if half else F32, dev)
        y = _empty((n * L, D), self.stack.dt, dev)
        mean1 = _empty((n * L,), F32, dev)
        rstd1 = _empty((n * L,), F32, dev)
        ln1 = self.stack.blocks[0].ln_1
        ops.vit_embed_ln(pe, v.class_embedding, v.positional_embedding, v.ln_pre.weight,
                         v.ln_pre.bias, ln1.weight, ln1.bias, x0, y, mean1, rstd1, n, npch)
        return x0, n, L, (y, mean1, rstd1)

    def forward_embedded(self, x0, n, L, save: bool, training: bool = False, prompts=None,
                         replace=None, first_ln1=None):
        """forward() from a precomputed embed() (the MVP query and prompt passes share x0)."""
        self._stage()
        last = None
        if x0.dtype == F16 and self.stack.variant == "adapter":
            # ln_post fused into the last block's adapter over every row
            v = self.visual
            M, D = x0.shape
            last = dict(w=v.ln_post.weight, b=v.ln_post.bias, y=_empty((M, D), BF16, x0.device),
                        mean=_empty((M,), F32, x0.device), rstd=_empty((M,), F32, x0.device))
        x, saved = self.stack.forward(x0, n, L, save, training, prompts=prompts, replace=replace,
                                      first_ln1=first_ln1, last_ln=last)
        if last is not None and last.get("done"):
            cls_idx = torch.arange(n, device=x.device, dtype=torch.int32) * L
            ci = cls_idx.long()
            lnp, mean, rstd = last["y"][ci], last["mean"][ci], last["rstd"][ci]
        else:
            lnp, cls_idx, mean, rstd = self._ln_post(x, n, L, self.stack.dt)
        f = _empty((n, self.projT.shape[0]), F32, x.device)
        ops.gemm_nt(lnp, self.projT, EPI_F32, f)
        ctx = dict(saved=saved, x=x, cls_idx=cls_idx, mean=mean, rstd=rstd, n=n, L=L,
                   prompt_layers=sorted(int(k) for k in (prompts or {}))) if save else None
        return f, ctx

    def backward(self, ctx, df, grads, on_layer=None, grad_stream=None, prompt_grads=None,
                 need_dx=False):
        """Returns the stack-input gradient (f32 [n*L, D]) when need_dx, else None."""
        v = self.visual
        dev = df.device
        n, L = ctx["n"], ctx["L"]
        D = v.width
        dt = self.stack.dt
        # the adapter and LoRA towers' half residual stream: its gradient in half as well (the
        # frozen prompt towers keep an f32 gradient: their prompt gradients are its rows)
        var = self.stack.variant
        half = ctx["x"].dtype == F16 and self.HALF_GRAD and (
            var == "adapter" or (var == "lora" and self.stack.lora_half_grad_ok()))
        gsc = sg = None
        out_grads, out_pg = grads, prompt_grads
        if half:
            # a per-call power-of-two gradient scale (the reference's GradScaler,
            # methods/adapter_clip.py:93): max|dL/df| lands in [2^12, 2^13), which keeps the
            # residual gradient (measured at <= 0.45 max|dL/df|, median 1e-4 of it) inside
            # half's normal range; the weight gradients divide it out
            df = df.contiguous().float().clone()
            if self._gsc is None or self._gsc.device != dev:
                self._gsc = torch.ones(1, dtype=F32, device=dev)
            gsc = self._gsc
            ops.grad_pow2_normalize(df, gsc, target_exp=self.GRAD_EXP)
        elif dt == F16:
            # the fp16 tower (f32 residual gradient, IEEE-half GEMM operands): the same scale,
            # with every returned gradient divided by it again (ScaledGrads)
            sg = ScaledGrads(self.stack, df, target_exp=self.GRAD_EXP)
            df, grads = sg.df, sg.grads
            prompt_grads = {} if prompt_grads is not None else None
        dfb = _empty(df.shape, dt, dev)
        ops.cast_bf16(df.contiguous(), dfb)
        dln = _empty((n, D), F32, dev)
        ops.gemm_nt(dfb, self.proj, EPI_F32, dln)
        dx, dxb = self._grad_in.get(n * L, D, dev, ctx["cls_idx"], key=(n, L),
                                    dt=dt, gdt=F16 if half else F32)
        if half and self.stack.half_grad_direct():
            dxb = None  # the adapter backward reads the half gradient itself (no bf16 copy)
        ops.layernorm_bwd(dln, ctx["x"], ctx["mean"], ctx["rstd"], v.ln_post.weight, dx, dxb,
                          row_idx=ctx["cls_idx"])
        # the input (patch embedding) is frozen; prompts appended at layer 0 need its backward
        gx, _ = self.stack.backward(ctx["saved"], dx, dxb, grads, n, L, on_layer, grad_stream,
                                    need_dx=need_dx or 0 in ctx["prompt_layers"],
                                    prompt_grads=prompt_grads, keep_input=True, gscale=gsc)
        if sg is not None:
            sg.add_to(out_grads)
            if out_pg is not None:
                for k, t in prompt_grads.items():
                    out_pg[k] = sg.unscaled(t)
            gx = sg.unscaled(gx)
        elif half and gx is not None:
            # the half residual gradient carries the scale: the f32 input gradient without it
            out = torch.zeros(gx.shape, dtype=F32, device=dev)
            ops.add_unscaled(out.view(-1), gx.float().contiguous().view(-1), gsc)
            gx = out
        return gx if need_dx else None


class TextTower:
    """CLIP.encode_text (model.py:941-956) on the engine."""

    def __init__(self, clip, stack: BlockStack):
        self.clip = clip
        self.stack = stack
        self._key = None
        self._grad_in = RowGrad()  # ln_final's backward writes the EOT rows only

    def _stage(self):
        c = self.clip
        key = _key(c.text_projection) + (self.stack.dt,)
        if key != self._key:
            P = c.text_projection
            dev = P.device
            self.projT = _empty((P.shape[1], P.shape[0]), self.stack.dt, dev)
            self.proj = _empty(tuple(P.shape), self.stack.dt, dev)
            ops.merge_weight(P.detach(), None, None, 0.0, self.proj, self.projT)
            self._key = key

    def forward(self, tokens, save: bool, training: bool = False, x0=None, replace=None):
        """tokens int64 [C, L] -> (features f32 [C, E], ctx). x0: optional precomputed input
        embeddings f32 [C*L, D] (token + positional; MaPLe's learned context rows,
        models/maple.py:40-45) — tokens then only locate the EOT rows; replace: row-replacing
        prompts per layer (BlockStack.forward)."""
        c = self.clip
        self._stage()
        dev = tokens.device
        tokens = tokens.contiguous().to(torch.int64)
        C, L = tokens.shape
        D = c.transformer.width
        if x0 is None:
            x0 = _empty((C * L, D), F32, dev)
            ops.text_embed(tokens, c.token_embedding.weight, c.positional_embedding, x0)
        x, saved = self.stack.forward(x0, C, L, save, training, replace=replace)
        eot = _empty((C,), torch.int32, dev)
        ops.eot_rows(tokens, eot)
        lnf = _empty((C, D), self.stack.dt, dev)
        mean = _empty((C,), F32, dev)
        rstd = _empty((C,), F32, dev)
        ops.layernorm_fwd(x, c.ln_final.weight, c.ln_final.bias, lnf, mean, rstd, row_idx=eot)
        f = _empty((C, self.projT.shape[0]), F32, dev)
        ops.gemm_nt(lnf, self.projT, EPI_F32, f)
        ctx = dict(saved=saved, x=x, eot=eot, mean=mean, rstd=rstd, C=C, L=L) if save else None
        return f, ctx

    def backward(self, ctx, df, grads, on_layer=None, prompt_grads=None, need_dx=False):
        """Returns the input-embedding gradient (f32 [C*L, D]) when need_dx, else None.

        IEEE-half storage (stack.set_storage(torch.float16)): the backward runs on a
        power-of-two-scaled incoming gradient and every gradient it returns (PEFT, prompt rows,
        input embeddings) is divided by that scale again (ScaledGrads)."""
        c = self.clip
        dev = df.device
        C, L = ctx["C"], ctx["L"]
        D = c.transformer.width
        dt = self.stack.dt
        sg = None
        df = df.contiguous()
        out_grads = grads
        if dt == F16:
            sg = ScaledGrads(self.stack, df)
            df, grads = sg.df, sg.grads
        dfb = _empty(df.shape, dt, dev)
        ops.cast_bf16(df, dfb)
        dln = _empty((C, D), F32, dev)
        ops.gemm_nt(dfb, self.proj, EPI_F32, dln)
        dx, dxb = self._grad_in.get(C * L, D, dev, ctx["eot"], dt=dt)
        ops.layernorm_bwd(dln, ctx["x"], ctx["mean"], ctx["rstd"], c.ln_final.weight, dx, dxb,
                          row_idx=ctx["eot"])
        pg = {} if (sg is not None and prompt_grads is not None) else prompt_grads
        gx, _ = self.stack.backward(ctx["saved"], dx, dxb, grads, C, L, on_layer,
                                    need_dx=need_dx, prompt_grads=pg, keep_input=True)
        if sg is not None:
            sg.add_to(out_grads)
            gx = sg.unscaled(gx)
            if prompt_grads is not None:
                for k, v in pg.items():
                    prompt_grads[k] = sg.unscaled(v)
        return gx
