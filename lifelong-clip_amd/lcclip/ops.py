"""Tensor-level wrappers over the C ABI (include/lc_clip.h). Shape/stride checks happen here and
again in the library; every call launches on torch's current stream of the tensor's device."""
from __future__ import annotations

import torch

from ._lib import call, ptr, stream_of

BF16 = torch.bfloat16
F16 = torch.float16
F32 = torch.float32
HALF = (BF16, F16)  # the 16-bit storage types (bf16: image tower; IEEE half: text tower)

EPI_BF16, EPI_F32, EPI_RESID, EPI_GELU, EPI_GELU_BWD, EPI_BF16_F32, EPI_GELU_D, EPI_MUL = range(8)
EPI_RESID16 = 14  # out0 / aux float16: the half residual stream (include/lc_clip.h)
EPI_GELU_D_Q8, EPI_MUL_Q8 = 12, 13  # gemm_nt_fp8 only: the result as the next fp8 GEMM's operand


def _rowmajor(t, dtype, name):
    if (t.dtype not in HALF) if dtype == HALF else (t.dtype != dtype):
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a 2-D row-major view, got shape {tuple(t.shape)} "
                         f"strides {t.stride()}")


def _sym16(name, *ts):
    """The entry point for the 16-bit storage type of `ts` (None and f32 entries ignored): `name`
    for bf16, `name`_f16 for IEEE half (include/lc_clip.h). The library reads raw pointers, so
    every 16-bit operand and output of one call must share the type: checked here."""
    kinds = {t.dtype for t in ts if t is not None and t.dtype in HALF}
    if len(kinds) > 1:
        raise TypeError(f"{name}: bf16 and float16 operands mixed in one call")
    return name + "_f16" if kinds == {F16} else name


SPLITK_TICKET_BYTES = 16384           # LC_SPLITK_TICKET_BYTES
SPLITK_WS_BYTES = SPLITK_TICKET_BYTES + 256 * 256 * 256 * 4   # tickets + 256 partial tiles
_workspaces = {}


def splitk_workspace(stream):
    """The split-K workspace of one HIP stream (launches on a stream are ordered, so they may
    share it): zeroed tickets + slab scratch, allocated from torch's caching allocator once."""
    key = (stream.device_index, stream.cuda_stream)
    ws = _workspaces.get(key)
    if ws is None:
        with torch.cuda.stream(stream):
            ws = torch.empty(SPLITK_WS_BYTES, dtype=torch.uint8, device=stream.device)
            ws[:SPLITK_TICKET_BYTES].zero_()
        _workspaces[key] = ws
    return ws


def gemm_nt(A, B, epi, out0, bias=None, alpha=1.0, out1=None, aux=None):
    """out = epilogue(alpha * A @ B^T + bias); A [M,K], B [N,K] bf16 (or both float16: the _f16
    entry point; 16-bit outputs / side inputs then float16 too). Large launches use the current
    stream's split-K workspace for their tail round (lc_gemm_nt_ws)."""
    _rowmajor(A, HALF, "A")
    _rowmajor(B, HALF, "B")
    if B.dtype != A.dtype:
        raise TypeError("gemm_nt: A and B must share the 16-bit type")
    M, K = A.shape
    N = B.shape[0]
    if B.shape[1] != K or out0.shape[0] != M or out0.shape[1] != N:
        raise ValueError(f"gemm_nt shapes A{tuple(A.shape)} B{tuple(B.shape)} out{tuple(out0.shape)}")
    if bias is not None and (bias.dtype != F32 or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("gemm_nt bias must be a contiguous f32 vector of length N")
    st = stream_of(A)
    ws = splitk_workspace(torch.cuda.current_stream(A.device)) if M >= 4096 else None
    name = "lc_gemm_nt_ws"
    if epi == EPI_RESID16:
        if A.dtype != BF16 or out0.dtype != F16 or aux is None or aux.dtype != F16 \
                or out0.stride(0) % 8 or aux.stride(0) % 8:
            raise TypeError("gemm_nt EPI_RESID16: bf16 operands, float16 out0 / aux (row stride % 8)")
    else:
        name = _sym16(name, A, out0, out1, aux)
    call(name, st, epi, M, N, K, ptr(A), A.stride(0), ptr(B), B.stride(0),
         ptr(bias), float(alpha), ptr(out0), out0.stride(0), ptr(out1),
         out1.stride(0) if out1 is not None else 0, ptr(aux), aux.stride(0) if aux is not None else 0,
         ptr(ws), ws.numel() if ws is not None else 0)
    return out0


# ------------------------------------------------------------------ block-scaled fp8 operands
FP8 = torch.uint8  # e4m3fn codes are carried as raw bytes


class Fp8Mat:
    """A [rows, K] e4m3 matrix in the fp8 GEMMs' operand format (lc_common.h): `data` uint8
    [rows, K] codes, `scales` uint8 [K/128, rows_pad, 4] E8M0 bytes (rows_pad = rows rounded up to
    256)."""
    __slots__ = ("data", "scales", "rows", "K")

    def __init__(self, rows, K, device, data=None, scales=None):
        if K % 128:
            raise ValueError("fp8 operands need K % 128 == 0")
        pad = (rows + 255) // 256 * 256
        self.rows, self.K = rows, K
        self.data = data if data is not None else torch.empty((rows, K), dtype=FP8, device=device)
        # rows >= `rows` of the scale buffer (the padding up to 256) carry no meaning: the GEMM
        # reads them only for tail rows it computes and never stores, and the branch-free
        # fp8-output GEMM epilogues (EPI_*_Q8) may write arbitrary bytes (0xFF included) there
        # from clamped tail rows. Only rows < `rows` are valid — never widen a narrow()ed view
        self.scales = scales if scales is not None else torch.empty((K // 128, pad, 4), dtype=FP8,
                                                                   device=device)

    @property
    def rows_pad(self):
        return self.scales.shape[1]

    def narrow(self, rows):
        """The first `rows` rows (a view; the scale buffer keeps its padded row count)."""
        out = Fp8Mat.__new__(Fp8Mat)
        out.data, out.scales, out.rows, out.K = self.data[:rows], self.scales, rows, self.K
        return out


def quant_fp8(src, out=None, transpose=False):
    """src [rows, K] bf16 or f32 (transpose=True: quantise src^T, i.e. along src's rows) ->
    Fp8Mat. Weights are quantised straight from their f32 master copy."""
    if src.dtype not in (BF16, F32) or src.dim() != 2:
        raise TypeError("quant_fp8: src must be a 2-D bf16 or f32 tensor")
    if transpose:
        K, rows = src.shape
        sr, sk = src.stride(1), src.stride(0)
    else:
        rows, K = src.shape
        sr, sk = src.stride(0), src.stride(1)
    if out is None:
        out = Fp8Mat(rows, K, src.device)
    if out.rows != rows or out.K != K:
        raise ValueError("quant_fp8: output shape mismatch")
    call("lc_quant_fp8", stream_of(src), rows, K, ptr(src), 1 if src.dtype == F32 else 0, sr, sk,
         ptr(out.data), out.data.stride(0), ptr(out.scales), out.rows_pad)
    return out


def gemm_nt_fp8(A, B, epi, out0, bias=None, alpha=1.0, out1=None, aux=None, q_out=None):
    """out = epilogue(alpha * A @ B^T + bias) with A, B Fp8Mat (block-scaled e4m3) on the fp8
    MFMA; epilogues as gemm_nt (BF16, F32, RESID, GELU, GELU_D, MUL), plus GELU_D_Q8 / MUL_Q8
    whose fp8 result (QuickGELU(pre) / alpha*acc*aux) goes to q_out, an Fp8Mat [M, N] — the same
    codes and scales as the bf16 epilogue followed by quant_fp8 (out0 is None for MUL_Q8)."""
    M, K = A.rows, A.K
    N = B.rows
    q8 = epi in (EPI_GELU_D_Q8, EPI_MUL_Q8)
    if B.K != K or (epi != EPI_MUL_Q8 and (out0.shape[0] != M or out0.shape[1] != N)):
        raise ValueError(f"gemm_nt_fp8 shapes A[{M},{K}] B[{N},{B.K}] out"
                         f"{None if out0 is None else tuple(out0.shape)}")
    if q8 and (q_out is None or q_out.rows != M or q_out.K != N):
        raise ValueError(f"gemm_nt_fp8: epilogue {epi} needs q_out Fp8Mat [{M}, {N}]")
    if bias is not None and (bias.dtype != F32 or bias.numel() != N or not bias.is_contiguous()):
        raise ValueError("gemm_nt_fp8 bias must be a contiguous f32 vector of length N")
    if epi == EPI_RESID16 and (out0.dtype != F16 or aux is None or aux.dtype != F16
                               or out0.stride(0) % 8 or aux.stride(0) % 8):
        raise TypeError("gemm_nt_fp8 EPI_RESID16: float16 out0 / aux (row stride % 8)")
    if q8:
        out1 = q_out.data
    st = stream_of(A.data)
    ws = splitk_workspace(torch.cuda.current_stream(A.data.device))
    call("lc_gemm_nt_fp8", st, epi, M, N, K, ptr(A.data), A.data.stride(0), ptr(A.scales),
         A.rows_pad, ptr(B.data), B.data.stride(0), ptr(B.scales), B.rows_pad, ptr(bias),
         float(alpha), ptr(out0), out0.stride(0) if out0 is not None else 0, ptr(out1),
         out1.stride(0) if out1 is not None else 0, ptr(aux), aux.stride(0) if aux is not None else 0,
         ptr(ws), ws.numel(), ptr(q_out.scales) if q8 else None, q_out.rows_pad if q8 else 0)
    return q_out if q8 else out0


def gemm_tn(A, B, C, alpha=1.0, colsum=None, colsum_scale=1.0):
    """C[N1,N2] += alpha * A[M,:N1]^T @ B[M,:N2] (C f32, N1 x N2 = C's shape); colsum[N1] +=
    colsum_scale * sum_m A[:, :N1]. A / B may be wider than N1 / N2 (zero padding to 64)."""
    _rowmajor(A, HALF, "A")
    _rowmajor(B, HALF, "B")
    _rowmajor(C, F32, "C")
    M = A.shape[0]
    N1, N2 = C.shape
    pad = lambda n: (n + 63) // 64 * 64  # noqa: E731
    # the kernel reads whole 64-column blocks of every row, the last row included
    if B.shape[0] != M or A.shape[1] < pad(N1) or B.shape[1] < pad(N2):
        raise ValueError("gemm_tn shape mismatch (operands must be readable to 64-column "
                         "multiples of C's shape)")
    if colsum is not None and (colsum.dtype != F32 or colsum.numel() != N1):
        raise ValueError("colsum must be f32 [N1]")
    # the launch stream's split-K workspace takes the two-stage partials (after its tickets)
    ws = splitk_workspace(torch.cuda.current_stream(A.device))
    call(_sym16("lc_gemm_tn_ws", A, B), stream_of(A), M, N1, N2, ptr(A), A.stride(0), ptr(B), B.stride(0),
         float(alpha), ptr(C), C.stride(0), ptr(colsum), float(colsum_scale), ptr(ws), ws.numel())
    return C


def _x16(name, x, *ts):
    """`name` for an f32 residual stream x, `name`_x16 for IEEE half x (the image tower's,
    include/lc_clip.h; bf16 / f32 partners only)."""
    if x.dtype == F32:
        return _sym16(name, *ts)
    if x.dtype != F16:
        raise TypeError(f"{name}: residual stream x must be f32 or float16, got {x.dtype}")
    if any(t is not None and t.dtype == F16 for t in ts):
        raise TypeError(f"{name}: a half residual stream takes bf16 / f32 partners")
    if x.stride(-1) != 1 or x.stride(0) % 4 or x.data_ptr() % 8:
        raise ValueError(f"{name}: half x must be row-major, 8-B aligned, row stride % 4 == 0")
    return name + "_x16"


def layernorm_fwd(x, weight, bias, y, mean=None, rstd=None, row_idx=None):
    """x: f32 or float16 (the image tower's half residual stream) [*, D]."""
    if x.dtype != F16:
        _rowmajor(x, F32, "x")
    rows = y.shape[0]
    D = x.shape[1]
    call(_x16("lc_layernorm_fwd", x, y), stream_of(x), rows, D, ptr(x), x.stride(0), ptr(row_idx),
         ptr(weight), ptr(bias), ptr(y), 1 if y.dtype == F32 else 0, y.stride(0), ptr(mean),
         ptr(rstd))
    return y


def layernorm_fwd_fp8(x, weight, bias, q, mean=None, rstd=None, y=None):
    """LayerNorm of x [rows, D] f32 (or float16: the half residual stream) straight into q, an
    Fp8Mat [rows, D] (the next fp8 GEMM's A operand; the codes of bf16 output + quant_fp8);
    y: optional bf16 copy."""
    if x.dtype != F16:
        _rowmajor(x, F32, "x")
    rows, D = x.shape
    if q.rows != rows or q.K != D or (y is not None and (y.dtype != BF16 or y.shape != x.shape)):
        raise ValueError("layernorm_fwd_fp8: output shape mismatch")
    call(_x16("lc_layernorm_fwd_fp8", x, y), stream_of(x), rows, D, ptr(x), x.stride(0), None, ptr(weight),
         ptr(bias), ptr(y), y.stride(0) if y is not None else 0, ptr(mean), ptr(rstd), ptr(q.data),
         q.data.stride(0), ptr(q.scales), q.rows_pad)
    return q


def layernorm_bwd(dy, x, mean, rstd, weight, dx, dx_bf16=None, dres=None, row_idx=None):
    """x: the forward's input, f32 or float16 (the half residual stream); dx (and dres): f32, or
    float16 with a half x (the half residual stream's gradient, lc_layernorm_bwd_g16)."""
    rows = dy.shape[0]
    D = x.shape[1]
    name = _x16("lc_layernorm_bwd", x, dy, dx_bf16)
    if dx.dtype == F16:
        if x.dtype != F16 or (dres is not None and dres.dtype != F16) or dx.stride(0) % 4 \
                or dx.data_ptr() % 8 or (dres is not None and dres.stride(0) != dx.stride(0)):
            raise ValueError("layernorm_bwd: a half gradient takes a half x and a half dres of "
                             "dx's row stride (% 4), 8-B aligned")
        name = "lc_layernorm_bwd_g16"
    elif dres is not None and dres.dtype != F32:
        raise TypeError("layernorm_bwd: dres must have dx's dtype")
    call(name, stream_of(x), rows, D, ptr(dy), 1 if dy.dtype == F32 else 0,
         dy.stride(0), ptr(x), x.stride(0), ptr(mean), ptr(rstd), ptr(weight), ptr(dres), ptr(dx),
         ptr(dx_bf16), dx.stride(0), ptr(row_idx))
    return dx


def layernorm_bwd_fp8(dy, x, mean, rstd, weight, dx, dx_bf16, q, dres=None):
    """layernorm_bwd whose result is also written into q, an Fp8Mat [rows, D]: the fp8 A operand
    of the next GEMM (the codes of dx_bf16 + quant_fp8). x f32 or float16 (the half residual
    stream; dx and dres stay f32)."""
    rows = dy.shape[0]
    D = x.shape[1]
    if q.rows != rows or q.K != D:
        raise ValueError("layernorm_bwd_fp8: output shape mismatch")
    if dx.dtype != F32 or (dres is not None and dres.dtype != F32):
        raise TypeError("layernorm_bwd_fp8: dx and dres are f32")
    call(_x16("lc_layernorm_bwd_fp8", x, dy, dx_bf16), stream_of(x), rows, D, ptr(dy), 1 if dy.dtype == F32 else 0,
         dy.stride(0), ptr(x), x.stride(0), ptr(mean), ptr(rstd), ptr(weight), ptr(dres), ptr(dx),
         ptr(dx_bf16), dx.stride(0), None, ptr(q.data), q.data.stride(0), ptr(q.scales), q.rows_pad)
    return q


def patchify(img, patch, out):
    """NCHW f32 images -> conv1's im2col rows, bf16 or float16 (out's type)."""
    if img.dtype != F32 or not img.is_contiguous():
        raise ValueError("patchify expects a contiguous f32 NCHW batch")
    n, c, h, w = img.shape
    if c != 3 or h != w:
        raise ValueError("patchify expects square 3-channel images")
    g = h // patch
    if out.dtype not in HALF or not out.is_contiguous() or out.numel() != n * g * g * 3 * patch * patch:
        raise ValueError("patchify: out must be contiguous bf16 / float16 [n*patches, 3*p*p]")
    call(_sym16("lc_patchify", out), stream_of(img), n, h, patch, ptr(img), ptr(out))
    return out


def vit_assemble(patch_emb, cls, pos, x, n_img, n_patch):
    call("lc_vit_assemble", stream_of(x), n_img, n_patch, x.shape[1], ptr(patch_emb), ptr(cls),
         ptr(pos), ptr(x))
    return x


def vit_embed_ln(patch_emb, cls, pos, ln_pre_w, ln_pre_b, ln1_w, ln1_b, x0, y, mean1, rstd1,
                 n_img, n_patch):
    """vit_assemble + ln_pre -> x0 (f32, or float16: the half residual stream) and the first
    block's ln_1 -> y (bf16), mean1, rstd1, in one launch (lc_vit_embed_ln[_x16])."""
    D = x0.shape[1]
    rows = n_img * (n_patch + 1)
    # y bf16, or float16 with an f32 x0 (the fp16 image tower: lc_vit_embed_ln_f16)
    if tuple(x0.shape) != (rows, D) or tuple(y.shape) != (rows, D) or x0.dtype not in (F32, F16) \
            or y.dtype not in ((BF16, F16) if x0.dtype == F32 else (BF16,)) \
            or not x0.is_contiguous() or not y.is_contiguous() \
            or tuple(patch_emb.shape) != (n_img * n_patch, D) or not patch_emb.is_contiguous():
        raise ValueError("vit_embed_ln: shape / layout mismatch")
    # every other operand is read raw by the kernel: f32, contiguous, of the sizes it assumes
    for name, t, numel in (("mean1", mean1, rows), ("rstd1", rstd1, rows), ("cls", cls, D),
                           ("pos", pos, (n_patch + 1) * D), ("ln_pre_w", ln_pre_w, D),
                           ("ln_pre_b", ln_pre_b, D), ("ln1_w", ln1_w, D), ("ln1_b", ln1_b, D)):
        if t.dtype != F32 or not t.is_contiguous() or t.numel() != numel or t.device != x0.device:
            raise ValueError(f"vit_embed_ln: {name} must be contiguous f32 with {numel} elements "
                             f"on {x0.device}")
    call(_x16("lc_vit_embed_ln", x0, y), stream_of(x0), n_img, n_patch, D, ptr(patch_emb), ptr(cls), ptr(pos),
         ptr(ln_pre_w), ptr(ln_pre_b), ptr(x0), ptr(ln1_w), ptr(ln1_b), ptr(y), ptr(mean1),
         ptr(rstd1))
    return x0


def text_embed(tokens, emb, pos, x):
    if tokens.dtype != torch.int64 or not tokens.is_contiguous():
        raise ValueError("tokens must be contiguous int64")
    C, L = tokens.shape
    call("lc_text_embed", stream_of(x), C, L, x.shape[1], ptr(tokens), ptr(emb), ptr(pos), ptr(x))
    return x


def eot_rows(tokens, out):
    C, L = tokens.shape
    call("lc_eot_rows", stream_of(tokens), C, L, ptr(tokens), ptr(out))
    return out


def attn_fwd(qkv, O, lse, n_seq, L, H, causal):
    if O.dtype != qkv.dtype or qkv.dtype not in HALF:
        raise TypeError("attn_fwd: qkv and O must share the 16-bit type")
    call(_sym16("lc_attn_fwd", qkv, O), stream_of(qkv), n_seq, L, H, ptr(qkv), qkv.stride(0), ptr(O), O.stride(0),
         ptr(lse), int(causal))
    return O


def attn_bwd(qkv, O, dO, lse, dqkv, n_seq, L, H, causal):
    if O.stride(0) != dO.stride(0):
        raise ValueError("O and dO must share a row stride")
    if len({t.dtype for t in (qkv, O, dO, dqkv)}) != 1 or qkv.dtype not in HALF:
        raise TypeError("attn_bwd: qkv, O, dO and dqkv must share the 16-bit type")
    call(_sym16("lc_attn_bwd", qkv, O, dO, dqkv), stream_of(qkv), n_seq, L, H, ptr(qkv), qkv.stride(0), ptr(O), ptr(dO),
         O.stride(0), ptr(lse), ptr(dqkv), dqkv.stride(0), int(causal))
    return dqkv


def attn_bwd_fp8(qkv, O, dO, lse, q, n_seq, L, H, causal):
    """attn_bwd with dq|dk|dv written straight into q, an Fp8Mat [n_seq*L, 3*H*64] (the fp8
    QKV input-gradient GEMM's A operand; the codes of attn_bwd + quant_fp8). L <= 224."""
    if O.stride(0) != dO.stride(0):
        raise ValueError("O and dO must share a row stride")
    if q.rows != n_seq * L or q.K != 3 * H * 64:
        raise ValueError("attn_bwd_fp8: output shape mismatch")
    call("lc_attn_bwd_fp8", stream_of(qkv), n_seq, L, H, ptr(qkv), qkv.stride(0), ptr(O), ptr(dO),
         O.stride(0), ptr(lse), ptr(q.data), q.data.stride(0), ptr(q.scales), q.rows_pad,
         int(causal))
    return q


def cast_bf16(src, dst):
    if src.dtype != F32 or not src.is_contiguous() or not dst.is_contiguous() or dst.dtype not in HALF:
        raise ValueError("cast_bf16 expects contiguous f32 -> bf16 / float16")
    call(_sym16("lc_cast_bf16", dst), stream_of(src), src.numel(), ptr(src), ptr(dst))
    return dst


def merge_weight(W, A, B, scaling, out, outT=None):
    """out = bf16(W + scaling * B @ A); A/B None -> plain cast."""
    N, K = W.shape
    r = 0 if A is None else A.shape[0]
    call(_sym16("lc_merge_weight", out, outT), stream_of(W), N, K, r, ptr(W), ptr(A), ptr(B), float(scaling),
         ptr(out), ptr(outT))
    return out


CAST_MAX = 64  # LC_CAST_MAX


def cast_weights(items):
    """items: [(W f32 [N, K], out bf16 [N, K], outT bf16 [K, N] or None)] -> one launch per
    CAST_MAX items (lc_cast_weights_bf16)."""
    import ctypes
    for i in range(0, len(items), CAST_MAX):
        chunk = items[i:i + CAST_MAX]
        n = len(chunk)
        for W, out, outT in chunk:
            if W.dtype != F32 or not W.is_contiguous() or out.dtype not in HALF or not out.is_contiguous():
                raise ValueError("cast_weights: W must be contiguous f32, out contiguous bf16 / float16")
            if out.shape != W.shape or (outT is not None and outT.shape != W.shape[::-1]):
                raise ValueError("cast_weights: shape mismatch")
        ws = (ctypes.c_void_p * n)(*[ptr(W) for W, _, _ in chunk])
        Ns = (ctypes.c_int * n)(*[W.shape[0] for W, _, _ in chunk])
        Ks = (ctypes.c_int * n)(*[W.shape[1] for W, _, _ in chunk])
        outs = (ctypes.c_void_p * n)(*[ptr(o) for _, o, _ in chunk])
        outTs = (ctypes.c_void_p * n)(*[ptr(t) for _, _, t in chunk])
        call(_sym16("lc_cast_weights_bf16", *[t for c in chunk for t in c[1:]]),
             stream_of(chunk[0][0]), n, ws, Ns, Ks, outs, outTs)


def merge_weights(items):
    """items: [(W f32 [N, K], A f32 [r, K] or None, B f32 [N, r] or None, scaling,
    out bf16 [N, K], outT bf16 [K, N] or None)] -> out = bf16(W + scaling B A) (and its
    transpose), one launch per CAST_MAX items (lc_merge_weights_bf16)."""
    import ctypes
    for i in range(0, len(items), CAST_MAX):
        chunk = items[i:i + CAST_MAX]
        n = len(chunk)
        for W, A, B, _, out, outT in chunk:
            if W.dtype != F32 or not W.is_contiguous() or out.dtype not in HALF or not out.is_contiguous():
                raise ValueError("merge_weights: W must be contiguous f32, out contiguous bf16 / float16")
            if out.shape != W.shape or (outT is not None and (outT.shape != W.shape[::-1]
                                                              or not outT.is_contiguous())):
                raise ValueError("merge_weights: shape mismatch")
            if A is not None:
                r = A.shape[0]
                if (A.dtype != F32 or B.dtype != F32 or not A.is_contiguous() or not B.is_contiguous()
                        or A.shape[1] != W.shape[1] or tuple(B.shape) != (W.shape[0], r) or r > 8):
                    raise ValueError("merge_weights: A [r, K] / B [N, r] f32 contiguous, r <= 8")
        P = ctypes.c_void_p
        ws = (P * n)(*[ptr(c[0]) for c in chunk])
        As = (P * n)(*[ptr(c[1]) for c in chunk])
        Bs = (P * n)(*[ptr(c[2]) for c in chunk])
        rs = (ctypes.c_int * n)(*[0 if c[1] is None else c[1].shape[0] for c in chunk])
        ss = (ctypes.c_float * n)(*[float(c[3]) for c in chunk])
        Ns = (ctypes.c_int * n)(*[c[0].shape[0] for c in chunk])
        Ks = (ctypes.c_int * n)(*[c[0].shape[1] for c in chunk])
        outs = (P * n)(*[ptr(c[4]) for c in chunk])
        outTs = (P * n)(*[ptr(c[5]) for c in chunk])
        call(_sym16("lc_merge_weights_bf16", *[t for c in chunk for t in c[4:]]),
             stream_of(chunk[0][0]), n, ws, As, Bs, rs, ss, Ns, Ks, outs,
             outTs)


def lora_grad(dY, X, A, B, scaling, dA, dB):
    M, N = dY.shape
    K = X.shape[1]
    call(_sym16("lc_lora_grad", dY, X), stream_of(dY), M, N, K, A.shape[0], ptr(dY), dY.stride(0), ptr(X),
         X.stride(0), ptr(A), ptr(B), float(scaling), ptr(dA), ptr(dB))


def lora_grad_1p(dY, X, a_pad, bt_pad, r, scaling, dA, dB, gscale=None):
    """dB [N,r] += s dY^T (X A^T), dA [r,K] += s (dY B)^T X in one pass over X and dY
    (lc_lora_grad_ws); a_pad [>=16, K] / bt_pad [>=16, N] bf16 with rows >= r zero. gscale:
    device f32 [1], the power-of-two scale dY carries (the half residual gradient), divided out
    (lc_lora_grad_ws_unscaled)."""
    _rowmajor(dY, HALF, "dY")
    _rowmajor(X, HALF, "X")
    _rowmajor(a_pad, HALF, "a_pad")
    _rowmajor(bt_pad, HALF, "bt_pad")
    M, N = dY.shape
    K = X.shape[1]
    if X.shape[0] != M or a_pad.shape[1] != K or bt_pad.shape[1] != N or a_pad.shape[0] < 16 \
            or bt_pad.shape[0] < 16 or tuple(dA.shape) != (r, K) or tuple(dB.shape) != (N, r):
        raise ValueError("lora_grad_1p: shape mismatch")
    # the kernel accumulates into dA / dB as dense row-major f32 (+=): anything else would be
    # silently corrupted. (The zero padding rows >= r of a_pad / bt_pad are the caller's
    # invariant: BlockStack._stage_lora allocates them zeroed and only ever writes rows < r.)
    for t, name in ((dA, "dA"), (dB, "dB")):
        if t.dtype != F32 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError(f"lora_grad_1p: {name} must be a contiguous f32 device tensor")
    ws = splitk_workspace(torch.cuda.current_stream(dY.device))
    name = _sym16("lc_lora_grad_ws", dY, X, a_pad, bt_pad)
    extra = ()
    if gscale is not None:
        if name != "lc_lora_grad_ws" or gscale.dtype != F32 or gscale.numel() != 1 \
                or not gscale.is_cuda:
            raise TypeError("lora_grad_1p: gscale is a device f32 [1] of the bf16 build")
        name, extra = "lc_lora_grad_ws_unscaled", (ptr(gscale),)
    call(name, stream_of(dY), M, N, K, r, ptr(dY), dY.stride(0), ptr(X), X.stride(0),
         ptr(a_pad), a_pad.stride(0), ptr(bt_pad), bt_pad.stride(0), float(scaling), ptr(dA),
         ptr(dB), ptr(ws), ws.numel(), *extra)


def adapter_fwd(z, Wd, bd, Wu, bu, scale, keep, seed, resid, xout, h, seed_dev=None):
    """xout = resid + z + scale * up(drop(relu(down(z)))): resid / xout f32 [M, D] (the kernel
    reads and writes them raw; a half residual stream goes through adapter_ln_fwd)."""
    M, D = z.shape
    if resid.dtype != F32 or xout.dtype != F32:
        raise TypeError("adapter_fwd: resid and xout must be f32")
    if tuple(resid.shape) != (M, D) or tuple(xout.shape) != (M, D) or resid.stride() != xout.stride() \
            or xout.stride(1) != 1:
        raise ValueError("adapter_fwd: resid and xout must be row-major [M, D] views of one stride")
    call(_sym16("lc_adapter_fwd", z, Wd, Wu, h), stream_of(z), M, D, ptr(z), z.stride(0), ptr(Wd), ptr(bd), ptr(Wu),
         ptr(bu), float(scale), float(keep), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev),
         ptr(resid), ptr(xout), xout.stride(0), ptr(h))


def adapter_ln_fwd(z, Wd, bd, Wu, bu, scale, keep, seed, resid, xout, h, gamma, beta, y, mean,
                   rstd, seed_dev=None):
    """adapter_fwd, then y = LayerNorm(xout) (bf16, statistics saved) in one launch. resid /
    xout: f32, or float16 (the image tower's half residual stream; xout row stride % 8 == 0)."""
    M, D = z.shape
    if y.dtype != z.dtype or tuple(y.shape) != (M, D) or y.stride(1) != 1:
        raise ValueError("adapter_ln_fwd: y must be a [M, D] row-major view of z's 16-bit type")
    if resid.dtype != xout.dtype or tuple(resid.shape) != (M, D) or tuple(xout.shape) != (M, D) \
            or resid.stride() != xout.stride():
        raise ValueError("adapter_ln_fwd: resid and xout must be [M, D] views of one dtype and stride")
    if xout.dtype == F16 and (xout.stride(0) % 8 or xout.data_ptr() % 16 or resid.data_ptr() % 16):
        raise ValueError("adapter_ln_fwd: half xout / resid rows must be 16-B aligned pieces")
    call(_x16("lc_adapter_ln_fwd", xout, z, Wd, Wu, h, y), stream_of(z), M, D, ptr(z), z.stride(0), ptr(Wd), ptr(bd), ptr(Wu),
         ptr(bu), float(scale), float(keep), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(seed_dev),
         ptr(resid), ptr(xout), xout.stride(0), ptr(h), ptr(gamma), ptr(beta), ptr(y),
         y.stride(0), ptr(mean), ptr(rstd))


def _g16(name, gout, *ts):
    """lc_adapter_*_g16 for a float16 gout beside bf16 partners (the image tower's half
    residual gradient, read directly: include/lc_clip.h), else the storage-type entry point."""
    if gout.dtype == F16 and any(t is not None and t.dtype == BF16 for t in ts):
        if any(t is not None and t.dtype == F16 for t in ts):
            raise TypeError(f"{name}: a float16 gout takes bf16 partners")
        if gout.stride(-1) != 1 or gout.stride(0) % 8 or gout.data_ptr() % 16:
            raise ValueError(f"{name}: half gout must be row-major, 16-B aligned, row stride % 8")
        return name + "_g16"
    return _sym16(name, gout, *ts)


def adapter_bwd(gout, h, WuT, WdT, scale, keep, dpre, dz):
    """dpre, dz (adapter.py:59-72 autograd). gout float16 with bf16 partners: the half residual
    gradient read directly (lc_adapter_bwd_g16, the same results as its bf16 copy)."""
    M, D = gout.shape
    call(_g16("lc_adapter_bwd", gout, h, WuT, WdT, dpre, dz), stream_of(gout), M, D, ptr(gout),
         gout.stride(0), ptr(h), ptr(WuT), ptr(WdT), float(scale), float(keep), ptr(dpre),
         ptr(dz), dz.stride(0) if dz is not None else D)


def adapter_wgrad(gout, h, z, dpre, scale, dWu, dbu, dWd, dbd, gscale=None):
    """dWu += scale gout^T h, dbu += scale colsum(gout), dWd += dpre^T z, dbd += colsum(dpre).
    gscale: optional device f32 scalar (a power-of-two gradient scale that gout / dpre carry):
    every result is divided by it (lc_adapter_wgrad_ws_unscaled)."""
    M, D = gout.shape
    for t, name in ((gout, "gout"), (z, "z")):
        _rowmajor(t, HALF, name)
    for t, name in ((h, "h"), (dpre, "dpre")):
        if t.dtype not in HALF or not t.is_contiguous() or t.shape != (M, 64):
            raise ValueError(f"{name} must be contiguous 16-bit [M, 64]")
    if z.shape != (M, D) or dWu.shape != (D, 64) or dWd.shape != (64, D):
        raise ValueError("adapter_wgrad shape mismatch")
    for t in (dWu, dWd, dbu, dbd):
        if t is not None and (t.dtype != F32 or not t.is_contiguous()):
            raise ValueError("gradient buffers must be contiguous f32")
    # two-stage reduction through the launch stream's split-K workspace (partials after its
    # ticket region; the stream orders every user of that buffer)
    ws = splitk_workspace(torch.cuda.current_stream(gout.device))
    if gscale is not None:
        # gout bf16, or float16 (the half residual gradient read directly: the _g16 form)
        name = _g16("lc_adapter_wgrad_ws_unscaled", gout, h, z, dpre)
        if (h.dtype != BF16 or z.dtype != BF16 or dpre.dtype != BF16 or gscale.dtype != F32
                or gscale.numel() != 1):
            raise TypeError("adapter_wgrad: gscale takes bf16 partners and an f32 device scalar")
        call(name, stream_of(gout), M, D, ptr(gout), gout.stride(0),
             ptr(h), ptr(z), z.stride(0), ptr(dpre), float(scale), ptr(dWu), ptr(dbu), ptr(dWd),
             ptr(dbd), ptr(ws), ws.numel(), ptr(gscale))
        return
    if gout.dtype != h.dtype:
        raise TypeError("adapter_wgrad: a float16 gout beside bf16 operands needs its gscale")
    call(_sym16("lc_adapter_wgrad_ws", gout, h, z, dpre), stream_of(gout), M, D, ptr(gout), gout.stride(0), ptr(h), ptr(z),
         z.stride(0), ptr(dpre), float(scale), ptr(dWu), ptr(dbu), ptr(dWd), ptr(dbd), ptr(ws),
         ws.numel())


def check_finite(g, flag):
    call("lc_check_finite", stream_of(g), g.numel(), ptr(g), ptr(flag))


def adamw(p, g, m, v, lr, b1, b2, eps, wd, step, skip=None, step_dev=None):
    call("lc_adamw", stream_of(p), p.numel(), ptr(p), ptr(g), ptr(m), ptr(v), float(lr), float(b1),
         float(b2), float(eps), float(wd), int(step), ptr(skip), ptr(step_dev))


def counter_add(ctr, delta=1):
    """ctr (int64 device tensor, <= 64 entries) += delta, on the current stream."""
    if ctr.dtype != torch.int64 or not ctr.is_contiguous():
        raise ValueError("counters must be a contiguous int64 tensor")
    call("lc_counter_add", stream_of(ctr), ctr.numel(), ptr(ctr), int(delta))


def adam_step_advance(ctr, skip=None):
    """ctr (int64 device scalar) += 1 unless skip[0] != 0: AdamW's step count advances only for
    applied updates (GradScaler skips optimizer.step() on non-finite gradients)."""
    if ctr.dtype != torch.int64 or ctr.numel() != 1:
        raise ValueError("the AdamW step counter must be one int64 element")
    call("lc_adam_step_advance", stream_of(ctr), ptr(ctr), ptr(skip))


def l2norm_rows(f, out, norms):
    R, E = f.shape
    call("lc_l2norm_rows", stream_of(f), R, E, ptr(f), f.stride(0), ptr(out), ptr(norms))


def clip_head(img_n, txt_n, logit_scale, labels, probs, dlogits, loss):
    B, E = img_n.shape
    C = txt_n.shape[0]
    call("lc_clip_head", stream_of(img_n), B, C, E, ptr(img_n), ptr(txt_n), ptr(logit_scale),
         ptr(labels), ptr(probs), ptr(dlogits), ptr(loss))


def head_logits(img_n, txt_n, logit_scale, logits, probs=None):
    B, E = img_n.shape
    C = txt_n.shape[0]
    call("lc_head_logits", stream_of(img_n), B, C, E, ptr(img_n), ptr(txt_n), ptr(logit_scale),
         ptr(logits), ptr(probs))


def softmax_bwd_rows(probs, dprobs, dlogits):
    B, C = probs.shape
    call("lc_softmax_bwd_rows", stream_of(probs), B, C, ptr(probs), ptr(dprobs), ptr(dlogits))


def head_feat_grad(dlogits, sr, sc, other_n, self_n, norms, logit_scale, dF, dn_ext=None):
    R, E = self_n.shape
    Co = other_n.shape[0]
    call("lc_head_feat_grad", stream_of(dlogits), R, Co, E, ptr(dlogits), sr, sc, ptr(other_n),
         ptr(self_n), ptr(norms), ptr(logit_scale), ptr(dn_ext), ptr(dF))


def grad_pow2_normalize(x, scale, target_exp=10):
    """x (contiguous f32) *= s in place, s = 2^(target_exp - floor(log2 max|x|)) on the device,
    written to scale (f32 [1]): the IEEE-half text tower's per-call loss scaling."""
    if x.dtype != F32 or not x.is_contiguous() or scale.dtype != F32 or scale.numel() < 1:
        raise ValueError("grad_pow2_normalize: contiguous f32 x and an f32 scale slot")
    call("lc_grad_pow2_normalize", stream_of(x), x.numel(), ptr(x), ptr(scale), int(target_exp))
    return x


def add_unscaled(y, x, scale):
    """y += x / scale[0] (contiguous f32, same size)."""
    if (y.dtype != F32 or x.dtype != F32 or not y.is_contiguous() or not x.is_contiguous()
            or y.numel() != x.numel()):
        raise ValueError("add_unscaled: contiguous f32 tensors of one size")
    call("lc_add_unscaled", stream_of(y), y.numel(), ptr(y), ptr(x), ptr(scale))
    return y


def device_cu_count(device):
    """Compute units of a HIP device (lc_device_cu_count)."""
    import ctypes
    n = ctypes.c_int(0)
    call("lc_device_cu_count", int(torch.device(device).index or 0), ctypes.byref(n))
    return n.value


class CUMaskedStream:
    """A HIP stream whose kernels run only on `count` CUs (first, first + stride, ...), wrapped
    as a torch.cuda.ExternalStream (lc_stream_create_cumask). The HIP stream lives as long as
    this object."""

    def __init__(self, device, count, stride=1, first=0):
        import ctypes
        dev = torch.device(device)
        h = ctypes.c_void_p(None)
        call("lc_stream_create_cumask", int(dev.index or 0), int(first), int(count), int(stride),
             ctypes.byref(h))
        self.handle = h.value
        self.count, self.stride, self.first = int(count), int(stride), int(first)
        self.stream = torch.cuda.ExternalStream(self.handle, device=dev)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                torch.cuda.synchronize()
                call("lc_stream_destroy", h)
            except Exception:
                pass
            self.handle = None
