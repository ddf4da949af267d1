"""Per-kernel parity on the MI355X: every HIP kernel vs a plain torch fp32 reference of the same op
evaluated on the same bf16-rounded inputs. Tolerances are stated per test: bf16 OUTPUTS carry a
rounding of 2^-9 relative, so bf16-output checks use a relative-norm bound of 4e-3 (fp32 outputs
1e-4); exact-integer tests catch layout bugs bit-exactly."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def ops(dev):
    from lcclip import ops as _ops
    return _ops


# ------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("M,N,K", [(300, 128, 64), (1000, 384, 768), (77, 192, 128),
                                   (4096, 768, 3072), (33, 64, 512)])
def test_gemm_nt_exact_integers(ops, dev, M, N, K):
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = torch.randint(-3, 4, (M, K), device=dev, generator=g).to(BF)
    B = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(BF)
    out = torch.empty(M, N, device=dev)
    ops.gemm_nt(A, B, ops.EPI_F32, out)
    ref = A.float() @ B.float().t()
    assert torch.equal(out, ref)


def test_gemm_qkv_dx_shape_on_hipblaslt(ops, dev):
    """The one step GEMM routed to hipBLASLt (blaslt.hip): the image tower's QKV input gradient
    at 256 images (M = 50 432, N = 768, K = 2 304, bf16 out, no bias), through ops.gemm_nt with
    its split-K workspace: exact on small integers (every partial sum is an integer below 2^24,
    so any summation order gives the same f32 and bf16-exact result), against torch fp32 on
    random data, and the same values as gemm8 (a forced tile keeps the hand-written kernel)."""
    from lcclip import _lib
    M, N, K = 50432, 768, 2304
    g = torch.Generator(device=dev).manual_seed(7)
    A = torch.randint(-2, 3, (M, K), device=dev, generator=g).to(BF)
    B = torch.randint(-2, 3, (N, K), device=dev, generator=g).to(BF)
    out = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_BF16, out)
    ref = A.float() @ B.float().t()
    assert torch.equal(out.float(), ref.to(BF).float())
    A = (torch.randn(M, K, device=dev, generator=g)).to(BF)
    B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(BF)
    ops.gemm_nt(A, B, ops.EPI_BF16, out)
    ref = A.float() @ B.float().t()
    assert rel(out, ref) < 4e-3
    lib = _lib.load()
    try:
        assert lib.lc_gemm_set_tile(8) == 0
        o8 = torch.empty_like(out)
        ops.gemm_nt(A, B, ops.EPI_BF16, o8)
    finally:
        lib.lc_gemm_set_tile(0)
    assert rel(out, o8) < 4e-3


@pytest.mark.parametrize("tile", [1, 2, 3, 5, 7, 8, 11])
def test_gemm_nt_every_tile_exact(ops, dev, tile):
    """Every tile kernel behind lc_gemm_nt (forced), ragged M, bit-exact on small integers, and
    the fused QuickGELU-derivative epilogue against torch at bf16 tolerance."""
    from lcclip import _lib
    lib = _lib.load()
    M, N, K = 4096 + 197, 512, 1024
    g = torch.Generator(device=dev).manual_seed(tile)
    A = torch.randint(-3, 4, (M, K), device=dev, generator=g).to(BF)
    B = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(BF)
    bias = torch.randint(-8, 9, (N,), device=dev, generator=g).float()
    out = torch.full((M, N), float("nan"), device=dev)
    gd = torch.empty(M, N, device=dev, dtype=BF)
    gl = torch.empty(M, N, device=dev, dtype=BF)
    Ar = torch.randn(M, K, device=dev).to(BF)
    Br = (torch.randn(N, K, device=dev) * K ** -0.5).to(BF)
    try:
        assert lib.lc_gemm_set_tile(tile) == 0
        ops.gemm_nt(A, B, ops.EPI_F32, out, bias=bias)
        ops.gemm_nt(Ar, Br, ops.EPI_GELU_D, gd, bias=bias, out1=gl)
    finally:
        lib.lc_gemm_set_tile(0)
    assert torch.equal(out, A.float() @ B.float().t() + bias)
    pre = Ar.float() @ Br.float().t() + bias
    s = torch.sigmoid(1.702 * pre)
    assert rel(gl, pre * s) < 4e-3
    assert rel(gd, s + 1.702 * pre * s * (1 - s)) < 4e-3


@pytest.mark.parametrize("M,N,K", [(1000, 384, 768), (77, 192, 128), (197 * 3, 2304, 768)])
def test_gemm_nt_epilogues(ops, dev, M, N, K):
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev).to(BF)
    B = (torch.randn(N, K, device=dev) * K ** -0.5).to(BF)
    bias = torch.randn(N, device=dev)
    ref = A.float() @ B.float().t() + bias
    o = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_BF16, o, bias=bias)
    assert rel(o, ref) < 4e-3
    o32 = torch.empty(M, N, device=dev)
    ops.gemm_nt(A, B, ops.EPI_F32, o32, bias=bias, alpha=1.0)
    assert rel(o32, ref) < 1e-5
    res = torch.randn(M, N, device=dev)
    ops.gemm_nt(A, B, ops.EPI_RESID, o32, bias=bias, aux=res)
    assert rel(o32, ref + res) < 1e-5
    pre = torch.empty(M, N, device=dev, dtype=BF)
    gl = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_GELU, pre, bias=bias, out1=gl)
    assert rel(pre, ref) < 4e-3
    assert rel(gl, ref * torch.sigmoid(1.702 * ref)) < 4e-3
    # GELU backward epilogue: out = (alpha * A B^T) * qgelu'(aux)
    aux = torch.randn(M, N, device=dev).to(BF)
    a = aux.float()
    s = torch.sigmoid(1.702 * a)
    dg = s + 1.702 * a * s * (1 - s)
    ob = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_GELU_BWD, ob, alpha=0.5, aux=aux)
    assert rel(ob, 0.5 * (A.float() @ B.float().t()) * dg) < 4e-3
    # derivative-saving forward epilogue and the multiply epilogue of its backward
    gd = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_GELU_D, gd, bias=bias, out1=gl)
    sr = torch.sigmoid(1.702 * ref)
    assert rel(gl, ref * sr) < 4e-3
    assert rel(gd, sr + 1.702 * ref * sr * (1 - sr)) < 4e-3
    om = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_MUL, om, alpha=0.5, aux=aux)
    assert rel(om, 0.5 * (A.float() @ B.float().t()) * a) < 4e-3
    # strided A view (row stride > K)
    Aw = torch.randn(M, K + 64, device=dev).to(BF)[:, 64:]
    ops.gemm_nt(Aw, B, ops.EPI_F32, o32)
    assert rel(o32, Aw.float() @ B.float().t()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(50432, 768, 3072), (50432, 768, 2304), (50432, 3072, 768),
                                   (296 * 256 - 100, 256, 2048), (50432, 768, 768),
                                   (12800, 768, 3072), (12800 - 37, 768, 2304)])
@pytest.mark.parametrize("tile", [0, 8])
def test_gemm_splitk_tail(ops, dev, M, N, K, tile):
    from lcclip import _lib
    lib = _lib.load()
    assert lib.lc_gemm_set_tile(tile) == 0
    try:
        _splitk_tail(ops, dev, M, N, K)
    finally:
        lib.lc_gemm_set_tile(0)


@pytest.mark.parametrize("M,N,K", [(50432, 768, 3072), (50432, 768, 2304), (50432 - 37, 768, 768),
                                   (25216, 768, 768), (296 * 256 - 100, 256, 2048)])
@pytest.mark.parametrize("mode", [2, 3, 4])
def test_gemm_streamk(ops, dev, M, N, K, mode):
    """Stream-K schedule of the 256x256 kernel (lc_gemm_set_streamk): equal (tile, k-tile) ranges
    per CU, tiles cut between two ranges summed through the workspace. Bit-exact on small
    integers (plain and residual epilogues), tickets left zero, deterministic on random data;
    mode 2 covers the N = 768 launches only (the N = 256 case then takes the split-K tail)."""
    from lcclip import _lib
    lib = _lib.load()
    assert lib.lc_gemm_set_streamk(mode) == 0
    assert lib.lc_gemm_set_streamk(5) != 0
    try:
        _splitk_tail(ops, dev, M, N, K)
        g = torch.Generator(device=dev).manual_seed(11)
        A = torch.randint(-3, 4, (M, K), device=dev, generator=g).to(BF)
        B = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(BF)
        res = torch.randint(-5, 6, (M, N), device=dev, generator=g).float()
        out = torch.full((M, N), float("nan"), device=dev)
        ops.gemm_nt(A, B, ops.EPI_RESID, out, aux=res)
        assert torch.equal(out, A.float() @ B.float().t() + res)
    finally:
        lib.lc_gemm_set_streamk(0)


def _splitk_tail(ops, dev, M, N, K):
    """The split-K tail of the 256x256 ping-pong GEMM (lc_gemm_nt_ws): these shapes leave the
    last round over 256 CUs at most half full (591 / 2364 / 296 tiles), so their tail tiles are
    summed from 3-4 K-slices; M = 12 800 (MaPLe's 64 images, 150 tiles: under one round) runs
    whole tiles (splitting every tile was measured slower: profiles/r03/sk_ab). Small integers: every partial sum is exact in f32, so the result
    must equal torch's bit for bit, for both the split and the plain (ws = NULL) launch; the
    fused epilogue must see the summed tile exactly once (bias added once)."""
    from lcclip._lib import call, ptr, stream_of
    g = torch.Generator(device=dev).manual_seed(7)
    A = torch.randint(-3, 4, (M, K), device=dev, generator=g).to(BF)
    B = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(BF)
    bias = torch.randint(-8, 9, (N,), device=dev, generator=g).float()
    ref = A.float() @ B.float().t() + bias
    out = torch.full((M, N), float("nan"), device=dev)
    ops.gemm_nt(A, B, ops.EPI_F32, out, bias=bias)  # M >= 4096: uses the stream's workspace
    assert torch.equal(out, ref)
    out2 = torch.full((M, N), float("nan"), device=dev)
    call("lc_gemm_nt_ws", stream_of(A), ops.EPI_F32, M, N, K, ptr(A), K, ptr(B), K, ptr(bias),
         1.0, ptr(out2), N, None, 0, None, 0, None, 0)
    assert torch.equal(out2, ref)
    # tickets are left zero for the next launch
    ws = ops.splitk_workspace(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    assert int(ws[:ops.SPLITK_TICKET_BYTES].sum()) == 0
    # bf16 epilogue on random data: deterministic across launches
    Ar = torch.randn(M, K, device=dev).to(BF)
    Br = (torch.randn(N, K, device=dev) * K ** -0.5).to(BF)
    o1 = torch.empty(M, N, device=dev, dtype=BF)
    o2 = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(Ar, Br, ops.EPI_BF16, o1, bias=bias)
    ops.gemm_nt(Ar, Br, ops.EPI_BF16, o2, bias=bias)
    assert torch.equal(o1, o2)
    assert rel(o1, Ar.float() @ Br.float().t() + bias) < 4e-3


def test_gemm_tail_rows_epilogues(ops, dev):
    """N = 3072, K = 768 at M = 50 432 (c_fc fwd / c_proj dX, 2364 tiles = 9.23 rounds): the
    two-output (QuickGELU, QuickGELU') and side-input (x aux) epilogues at full size, checked at
    the first rows, across the 9-round boundary and in the last partial round, against torch."""
    torch.manual_seed(3)
    M, N, K = 50432, 3072, 768
    A = torch.randn(M, K, device=dev).to(BF)
    B = (torch.randn(N, K, device=dev) * K ** -0.5).to(BF)
    bias = torch.randn(N, device=dev)
    gd = torch.empty(M, N, device=dev, dtype=BF)
    gl = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_GELU_D, gd, bias=bias, out1=gl)
    aux = torch.randn(M, N, device=dev).to(BF)
    om = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt(A, B, ops.EPI_MUL, om, alpha=0.5, aux=aux)
    for lo, hi in ((0, 512), (49152 - 256, 49152 + 256), (M - 700, M)):
        ref = A[lo:hi].float() @ B.float().t()
        pre = ref + bias
        sr = torch.sigmoid(1.702 * pre)
        assert rel(gl[lo:hi], pre * sr) < 4e-3
        assert rel(gd[lo:hi], sr + 1.702 * pre * sr * (1 - sr)) < 4e-3
        assert rel(om[lo:hi], 0.5 * ref * aux[lo:hi].float()) < 4e-3


@pytest.mark.parametrize("M,N1,N2", [(100, 128, 64), (3000, 64, 768), (50432 // 8, 768, 64)])
def test_gemm_tn(ops, dev, M, N1, N2):
    torch.manual_seed(1)
    A = torch.randn(M, N1, device=dev).to(BF)
    B = torch.randn(M, N2, device=dev).to(BF)
    C = torch.ones(N1, N2, device=dev)
    cs = torch.ones(N1, device=dev)
    ops.gemm_tn(A, B, C, alpha=0.5, colsum=cs, colsum_scale=0.25)
    ref = 1 + 0.5 * A.float().t() @ B.float()
    assert rel(C - 1, ref - 1) < 1e-5
    assert rel(cs - 1, 0.25 * A.float().sum(0)) < 1e-5


@pytest.mark.parametrize("M,D", [(77 * 10, 512), (50432 // 8 + 37, 768)])
def test_adapter_wgrad(ops, dev, M, D):
    """Both adapter weight/bias gradients in one launch (ragged M: masked last step)."""
    torch.manual_seed(5)
    gout = torch.randn(M, D, device=dev).to(BF)
    z = torch.randn(M, D, device=dev).to(BF)
    h = torch.randn(M, 64, device=dev).to(BF)
    dpre = torch.randn(M, 64, device=dev).to(BF)
    dWu = torch.full((D, 64), 2.0, device=dev)
    dbu = torch.full((D,), 2.0, device=dev)
    dWd = torch.full((64, D), 2.0, device=dev)
    dbd = torch.full((64,), 2.0, device=dev)
    ops.adapter_wgrad(gout, h, z, dpre, 0.1, dWu, dbu, dWd, dbd)  # two-stage (workspace)
    assert rel(dWu - 2, 0.1 * gout.float().t() @ h.float()) < 1e-5
    assert rel(dbu - 2, 0.1 * gout.float().sum(0)) < 1e-5
    assert rel(dWd - 2, dpre.float().t() @ z.float()) < 1e-5
    assert rel(dbd - 2, dpre.float().sum(0)) < 1e-5
    # the single-stage form (f32 atomics, no workspace) on the same inputs
    from lcclip._lib import call, ptr, stream_of
    out = [torch.full_like(t, 2.0) for t in (dWu, dbu, dWd, dbd)]
    call("lc_adapter_wgrad", stream_of(gout), M, D, ptr(gout), gout.stride(0), ptr(h), ptr(z),
         z.stride(0), ptr(dpre), 0.1, *[ptr(t) for t in out])
    for a, b in zip(out, (dWu, dbu, dWd, dbd)):
        assert rel(a - 2, b - 2) < 1e-6


def test_gemm_tn_masked_rank4(ops, dev):
    """N1 or N2 below 64 (zero-padded [M,64] operands, outputs masked): the LoRA dA / dB path."""
    torch.manual_seed(11)
    M, N, r = 3000, 2304, 4
    dY = torch.randn(M, N, device=dev).to(BF)
    xa = torch.zeros(M, 64, device=dev, dtype=BF)
    xa[:, :r] = torch.randn(M, r, device=dev).to(BF)
    dB = torch.ones(N, r, device=dev)
    ops.gemm_tn(dY, xa, dB, alpha=0.25)
    assert rel(dB - 1, 0.25 * dY.float().t() @ xa[:, :r].float()) < 1e-5
    X = torch.randn(M, 768, device=dev).to(BF)
    dA = torch.zeros(r, 768, device=dev)
    ops.gemm_tn(xa, X, dA, alpha=2.0)
    assert rel(dA, 2.0 * xa[:, :r].float().t() @ X.float()) < 1e-5


# ------------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("D", [64, 128, 512, 768])
def test_layernorm_fwd_bwd(ops, dev, D):
    torch.manual_seed(2)
    R = 333
    x = torch.randn(R, D, device=dev) * 3 + 1
    w = torch.randn(D, device=dev)
    b = torch.randn(D, device=dev)
    y = torch.empty(R, D, device=dev, dtype=BF)
    mean = torch.empty(R, device=dev)
    rstd = torch.empty(R, device=dev)
    ops.layernorm_fwd(x, w, b, y, mean, rstd)
    xr = x.clone().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xr, (D,), w, b, 1e-5)
    assert rel(y, ref) < 4e-3
    y32 = torch.empty(R, D, device=dev)
    ops.layernorm_fwd(x, w, b, y32)
    assert rel(y32, ref) < 1e-5
    dy = torch.randn(R, D, device=dev).to(BF)
    ref.backward(dy.float())
    dres = torch.randn(R, D, device=dev)
    dx = torch.empty(R, D, device=dev)
    dxb = torch.empty(R, D, device=dev, dtype=BF)
    ops.layernorm_bwd(dy, x, mean, rstd, w, dx, dxb, dres=dres)
    assert rel(dx, xr.grad + dres) < 1e-4
    assert rel(dxb, xr.grad + dres) < 4e-3
    # gathered rows (ln_post on CLS rows / ln_final on EOT rows)
    idx = torch.tensor([0, 17, 34, 200], device=dev, dtype=torch.int32)
    yg = torch.empty(4, D, device=dev)
    mg = torch.empty(4, device=dev)
    rg = torch.empty(4, device=dev)
    ops.layernorm_fwd(x, w, b, yg, mg, rg, row_idx=idx)
    assert rel(yg, ref.detach()[idx.long()]) < 1e-5
    dyg = torch.randn(4, D, device=dev)
    dxg = torch.zeros(R, D, device=dev)
    ops.layernorm_bwd(dyg, x, mg, rg, w, dxg, None, row_idx=idx)
    xr2 = x[idx.long()].clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xr2, (D,), w, b, 1e-5).backward(dyg)
    assert rel(dxg[idx.long()], xr2.grad) < 1e-4
    assert dxg.abs().sum() == dxg[idx.long()].abs().sum()


# ------------------------------------------------------------------------------- attention
def ref_attention(q, k, v, causal):
    s = (q @ k.transpose(-1, -2)) * 0.125
    if causal:
        L = s.shape[-1]
        s = s + torch.full((L, L), float("-inf"), device=s.device).triu_(1)
    return torch.softmax(s, -1) @ v


@pytest.mark.parametrize("n,L,H,causal", [(3, 17, 2, False), (4, 77, 8, True), (2, 197, 12, False),
                                          (5, 32, 1, True), (2, 200, 2, False), (3, 224, 2, False),
                                          (2, 256, 2, True), (1, 250, 3, False),
                                          (2, 213, 3, True), (1, 193, 2, False)])
def test_attention_fwd_bwd(ops, dev, n, L, H, causal):
    torch.manual_seed(3)
    D = H * 64
    qkv = (torch.randn(n * L, 3 * D, device=dev) * 1.5).to(BF)
    O = torch.empty(n * L, D, device=dev, dtype=BF)
    lse = torch.empty(n * H, L, device=dev)
    ops.attn_fwd(qkv, O, lse, n, L, H, causal)
    t = qkv.float().reshape(n, L, 3, H, 64).permute(2, 0, 3, 1, 4)  # 3, n, H, L, 64
    q, k, v = (x.clone().requires_grad_(True) for x in t)
    ref = ref_attention(q, k, v, causal)
    got = O.float().reshape(n, L, H, 64).permute(0, 2, 1, 3)
    assert rel(got, ref) < 8e-3
    s = (q @ k.transpose(-1, -2)) * 0.125
    if causal:
        s = s + torch.full((L, L), float("-inf"), device=dev).triu_(1)
    ref_lse = torch.logsumexp(s, -1) / math.log(2)
    assert rel(lse.reshape(n, H, L), ref_lse) < 1e-4
    dO = torch.randn(n * L, D, device=dev).to(BF)
    dqkv = torch.empty(n * L, 3 * D, device=dev, dtype=BF)
    ops.attn_bwd(qkv, O, dO, lse, dqkv, n, L, H, causal)
    # reference gradient through the attention actually computed (its O is the bf16 one)
    ref.backward(dO.float().reshape(n, L, H, 64).permute(0, 2, 1, 3))
    g = dqkv.float().reshape(n, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    assert rel(g[0], q.grad) < 2e-2
    assert rel(g[1], k.grad) < 2e-2
    assert rel(g[2], v.grad) < 2e-2


@pytest.mark.parametrize("n,L,H,causal", [(3, 17, 2, False), (4, 77, 8, True), (2, 197, 12, False),
                                          (5, 32, 1, True), (2, 200, 2, False), (3, 224, 2, False),
                                          (2, 213, 3, True), (1, 193, 2, False), (2, 202, 2, False),
                                          (1, 250, 2, False), (3, 100, 2, True)])
def test_attention_bwd_forms(ops, dev, n, L, H, causal):
    """Every lc_attn_bwd form (lc_attn_bwd_set_form: 1 fused dS^T park, 2 key-major + query-major
    pair, 3 two-phase at two workgroups per CU) against the torch fp32 gradient of the attention
    actually computed, and against each other: the same bf16 dS / P operands, so they differ only
    where an f32 sum order flips a bf16 rounding (lora.py:1043-1068 autograd)."""
    from lcclip import _lib
    torch.manual_seed(5)
    D = H * 64
    lib = _lib.load()
    qkv = (torch.randn(n * L, 3 * D, device=dev) * 1.5).to(BF)
    O = torch.empty(n * L, D, device=dev, dtype=BF)
    lse = torch.empty(n * H, L, device=dev)
    ops.attn_fwd(qkv, O, lse, n, L, H, causal)
    t = qkv.float().reshape(n, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    q, k, v = (x.clone().requires_grad_(True) for x in t)
    dO = torch.randn(n * L, D, device=dev).to(BF)
    ref_attention(q, k, v, causal).backward(dO.float().reshape(n, L, H, 64).permute(0, 2, 1, 3))
    outs = {}
    try:
        for form in (1, 2, 3):
            assert lib.lc_attn_bwd_set_form(form) == 0
            dqkv = torch.full((n * L, 3 * D), float("nan"), device=dev, dtype=BF)
            ops.attn_bwd(qkv, O, dO, lse, dqkv, n, L, H, causal)
            torch.cuda.synchronize()
            g = dqkv.float().reshape(n, L, 3, H, 64).permute(2, 0, 3, 1, 4)
            assert torch.isfinite(g).all(), form
            for i, ref in enumerate((q.grad, k.grad, v.grad)):
                assert rel(g[i], ref) < 2e-2, (form, i)
            outs[form] = g
    finally:
        lib.lc_attn_bwd_set_form(0)
    assert lib.lc_attn_bwd_set_form(4) != 0
    for form in (2, 3):
        for i in range(3):
            assert rel(outs[form][i], outs[1][i]) < 4e-3, (form, i)


# ------------------------------------------------------------------------------- train transform
@pytest.mark.parametrize("params", [(0, 0, False), (8, 8, True), (3, 5, True), (4, 4, False)])
def test_train_transform_vs_oracle(dev, params):
    """lc_train_transform (methods/_trainer.py:212-242 minus the AutoAugment op) vs the oracle's
    torch restatement on CIFAR-shaped ToTensor batches: f32 NCHW within 2e-6 absolute (the
    bilinear taps are summed in a different order, normalise as one FMA), the fused bf16 patch layout equal to
    patchify(oracle) up to one bf16 rounding step."""
    import oracle.clip_oracle as o
    from lcclip.transforms import TrainTransform
    i, j, flip = params
    g = torch.Generator().manual_seed(sum(params) + 1)
    x = torch.randint(0, 256, (6, 3, 32, 32), generator=g).float() / 255  # ToTensor values
    tf = TrainTransform.for_dataset("cifar100")
    ref = o.train_transform(x, 224, 4, i, j, flip, tf.mean, tf.std, quantize=True)
    got = tf(x.to(dev), params=params)
    assert got.shape == (6, 3, 224, 224)
    assert (got.cpu() - ref).abs().max().item() < 2e-6
    pt = tf(x.to(dev), params=params, layout="patches")
    pref = o.patchify(ref, 16)
    assert pt.shape == (6 * 196, 768) and pt.dtype == BF
    d = (pt.float().cpu() - pref).abs()
    assert (d <= pref.abs() * 2 ** -7 + 1e-6).all()
    # a same-size resize with identity normalisation isolates the uint8 round trip (and the
    # flip): the kernel equals torch bit for bit, with and without the quantisation
    for q in (False, True):
        tf2 = TrainTransform((0.0,) * 3, (1.0,) * 3, inp_size=32, padding=0, autoaug=q)
        ref2 = o.train_transform(x, 32, 0, 0, 0, flip, tf2.mean, tf2.std, quantize=q)
        assert torch.equal(tf2(x.to(dev), params=(0, 0, flip)).cpu(), ref2)


def test_train_transform_large_input_path(dev):
    """Inputs too large for the LDS-staged kernel (3 x 96 x 96 f32 > 64 KiB) take the gather
    kernel: same oracle bound, both layouts."""
    import oracle.clip_oracle as o
    from lcclip.transforms import TrainTransform
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 256, (3, 3, 96, 96), generator=g).float() / 255
    tf = TrainTransform.for_dataset("imagenet-r")
    ref = o.train_transform(x, 224, 4, 6, 1, True, tf.mean, tf.std, quantize=True)
    got = tf(x.to(dev), params=(6, 1, True))
    assert (got.cpu() - ref).abs().max().item() < 2e-6
    pt = tf(x.to(dev), params=(6, 1, True), layout="patches")
    pref = o.patchify(ref, 16)
    assert ((pt.float().cpu() - pref).abs() <= pref.abs() * 2 ** -7 + 1e-6).all()


def test_transform_patches_feed_the_image_tower(dev):
    """The fused patch layout is a drop-in input of the image tower: same features as the f32
    image batch through lc_patchify."""
    from lcclip import AdapterCLIP
    from lcclip.transforms import TrainTransform
    torch.manual_seed(0)
    w = AdapterCLIP("ViT-B/16", peft_method="adapter", peft_encoder="both", device=dev)
    x = (torch.randint(0, 256, (4, 3, 32, 32), device=dev).float() / 255)
    tf = TrainTransform.for_dataset("cifar100")
    prm = tf.draw()
    with torch.no_grad():
        f_img = w.encode_image(tf(x, params=prm))
        f_pt = w.encode_image(tf(x, params=prm, layout="patches"))
    assert rel(f_pt, f_img) < 1e-6


# ------------------------------------------------------------------------------- PEFT
@pytest.mark.parametrize("D,M,keep", [(768, 1000, 1.0), (128, 77, 1.0), (512, 300, 0.9),
                                      (768, 4109, 0.9), (512, 2000, 1.0)])
def test_adapter_fwd_bwd(ops, dev, D, M, keep):
    torch.manual_seed(4)
    z = torch.randn(M, D, device=dev).to(BF)
    Wd = (torch.randn(64, D, device=dev) * D ** -0.5).to(BF)
    bd = torch.randn(64, device=dev) * 0.1
    Wu = (torch.randn(D, 64, device=dev) * 0.125).to(BF)
    bu = torch.randn(D, device=dev) * 0.1
    resid = torch.randn(M, D, device=dev)
    x = torch.empty(M, D, device=dev)
    h = torch.empty(M, 64, device=dev, dtype=BF)
    ops.adapter_fwd(z, Wd, bd, Wu, bu, 0.1, keep, 1234, resid, x, h)
    hr = torch.relu(z.float() @ Wd.float().t() + bd)
    if keep < 1.0:
        kept = h.float() > 0
        assert (kept <= (hr > 0)).all()
        frac = kept[hr > 0].float().mean().item()
        assert abs(frac - keep) < 0.03  # dropout keep rate
        hr = torch.where(kept, hr / keep, torch.zeros_like(hr))
    assert rel(h, hr) < 4e-3
    ref = resid + z.float() + 0.1 * (h.float() @ Wu.float().t() + bu)
    assert rel(x, ref) < 1e-4
    # backward
    g = torch.randn(M, D, device=dev).to(BF)
    dpre = torch.empty(M, 64, device=dev, dtype=BF)
    dz = torch.empty(M, D, device=dev, dtype=BF)
    ops.adapter_bwd(g, h, Wu.t().contiguous(), Wd.t().contiguous(), 0.1, keep, dpre, dz)
    dh = 0.1 * g.float() @ Wu.float()
    dpr = torch.where(h.float() > 0, dh / keep, torch.zeros_like(dh))
    assert rel(dpre, dpr) < 4e-3
    assert rel(dz, g.float() + dpre.float() @ Wd.float()) < 4e-3


@pytest.mark.parametrize("D,M,with_dz", [(768, 50432, True), (768, 4109, True), (768, 1031, True),
                                         (512, 2013, True), (768, 4109, False)])
def test_adapter_bwd_fused_matches_gemms(ops, dev, D, M, with_dz):
    """The one-pass adapter backward (row-block walker, M >= 1024 at D = 768 / 512) gives the
    two-GEMM form's dpre and dz bit for bit (same MFMA operand and k order, same epilogue
    arithmetic): ragged last block, a walker with a single block, the step's row count; and the
    dpre-only call (routed to the GEMM either way)."""
    torch.manual_seed(D + M)
    g = torch.randn(M, D, device=dev).to(BF)
    h = torch.relu(torch.randn(M, 64, device=dev)).to(BF)
    Wu = (torch.randn(D, 64, device=dev) * 0.125).to(BF)
    Wd = (torch.randn(64, D, device=dev) * D ** -0.5).to(BF)
    WuT, WdT = Wu.t().contiguous(), Wd.t().contiguous()
    outs = {}
    from lcclip import _lib
    lib = _lib.load()
    try:
        for mode in ("1", "0"):
            lib.lc_adapter_bwd_set_form(int(mode))
            dpre = torch.full((M, 64), 7.0, device=dev, dtype=BF)
            dz = torch.full((M, D), 7.0, device=dev, dtype=BF) if with_dz else None
            ops.adapter_bwd(g, h, WuT, WdT, 0.1, 0.9, dpre, dz)
            torch.cuda.synchronize()
            outs[mode] = (dpre, dz)
    finally:
        lib.lc_adapter_bwd_set_form(1)  # process-wide: restored even if a launch raised
    assert torch.equal(outs["1"][0], outs["0"][0])
    if with_dz:
        assert torch.equal(outs["1"][1], outs["0"][1])


def test_lora_merge_and_grad(ops, dev):
    torch.manual_seed(5)
    N, K, r, M = 2304, 768, 4, 2000
    W = torch.randn(N, K, device=dev)
    A = torch.randn(r, K, device=dev)
    B = torch.randn(N, r, device=dev)
    out = torch.empty(N, K, device=dev, dtype=BF)
    outT = torch.empty(K, N, device=dev, dtype=BF)
    ops.merge_weight(W, A, B, 0.25, out, outT)
    ref = W + 0.25 * B @ A
    assert rel(out, ref) < 4e-3
    assert torch.equal(outT, out.t())
    # ragged shapes (edge tiles, scalar paths) and the padded-operand staging uses (r = 0)
    for n_, k_, r_ in [(100, 70, 4), (2304, 4, 0), (4, 768, 0), (77, 131, 3)]:
        W2 = torch.randn(n_, k_, device=dev)
        A2, B2 = torch.randn(r_, k_, device=dev), torch.randn(n_, r_, device=dev)
        o2 = torch.empty(n_, k_, device=dev, dtype=BF)
        o2T = torch.empty(k_, n_, device=dev, dtype=BF)
        ops.merge_weight(W2, A2 if r_ else None, B2 if r_ else None, 0.5, o2, o2T)
        assert rel(o2, W2 + 0.5 * B2 @ A2) < 4e-3
        assert torch.equal(o2T, o2.t())
    dY = torch.randn(M, N, device=dev).to(BF)
    X = torch.randn(M, K, device=dev).to(BF)
    dA = torch.zeros(r, K, device=dev)
    dB = torch.zeros(N, r, device=dev)
    ops.lora_grad(dY, X, A, B, 0.25, dA, dB)
    assert rel(dB, 0.25 * dY.float().t() @ (X.float() @ A.t())) < 1e-4
    assert rel(dA, 0.25 * (dY.float() @ B).t() @ X.float()) < 1e-4


def test_adamw_matches_torch(ops, dev):
    torch.manual_seed(6)
    n = 10007
    p = torch.randn(n, device=dev)
    q = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([q], lr=5e-4, weight_decay=1e-5)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    skip = torch.zeros(1, device=dev, dtype=torch.int32)
    for step in range(1, 4):
        g = torch.randn(n, device=dev)
        q.grad = g.clone()
        opt.step()
        ops.check_finite(g, skip)
        ops.adamw(p, g, m, v, 5e-4, 0.9, 0.999, 1e-8, 1e-5, step, skip)
    assert rel(p, q.detach()) < 1e-6
    g[5] = float("inf")
    before = p.clone()
    ops.check_finite(g, skip)
    ops.adamw(p, g, m, v, 5e-4, 0.9, 0.999, 1e-8, 1e-5, 4, skip)
    assert skip.item() == 1 and torch.equal(p, before)  # GradScaler-style skip


# ------------------------------------------------------------------------------- embeddings
def test_patchify_assemble_text_embed(ops, dev):
    torch.manual_seed(7)
    n, res, P, D = 3, 64, 16, 128
    img = torch.randn(n, 3, res, res, device=dev)
    g = res // P
    patches = torch.empty(n * g * g, 3 * P * P, device=dev, dtype=BF)
    ops.patchify(img, P, patches)
    ref = img.reshape(n, 3, g, P, g, P).permute(0, 2, 4, 1, 3, 5).reshape(n * g * g, -1)
    assert torch.equal(patches, ref.to(BF))
    pe = torch.randn(n * g * g, D, device=dev)
    cls = torch.randn(D, device=dev)
    pos = torch.randn(g * g + 1, D, device=dev)
    x = torch.empty(n * (g * g + 1), D, device=dev)
    ops.vit_assemble(pe, cls, pos, x, n, g * g)
    refx = torch.cat([cls.expand(n, 1, D), pe.reshape(n, g * g, D)], 1) + pos
    assert torch.equal(x, refx.reshape(-1, D))
    C, L, V = 5, 77, 512
    tok = torch.randint(0, 500, (C, L), device=dev)
    tok[torch.arange(C), torch.tensor([3, 9, 76, 0, 40])] = 511
    emb = torch.randn(V, D, device=dev)
    posT = torch.randn(L, D, device=dev)
    xt = torch.empty(C * L, D, device=dev)
    ops.text_embed(tok, emb, posT, xt)
    assert torch.equal(xt, (emb[tok] + posT).reshape(-1, D))
    eot = torch.empty(C, device=dev, dtype=torch.int32)
    ops.eot_rows(tok, eot)
    assert eot.tolist() == [c * L + t for c, t in enumerate(tok.argmax(-1).tolist())]


# ------------------------------------------------------------------------------- head
@pytest.mark.parametrize("B,C", [(2, 3), (256, 10), (64, 200)])
def test_head_fused_and_module_kernels(ops, dev, B, C):
    torch.manual_seed(8)
    E = 512
    fi = torch.randn(B, E, device=dev)
    ft = torch.randn(C, E, device=dev)
    ls = torch.tensor([math.log(1 / 0.07)], device=dev)
    y = torch.randint(0, C, (B,), device=dev)
    fir, ftr = fi.clone().requires_grad_(True), ft.clone().requires_grad_(True)
    i_n = fir / fir.norm(dim=-1, keepdim=True)
    t_n = ftr / ftr.norm(dim=-1, keepdim=True)
    logits = ls.exp() * i_n @ t_n.t()
    probs_ref = logits.softmax(-1)
    loss_ref = torch.nn.functional.cross_entropy(probs_ref, y)
    loss_ref.backward()
    img_n = torch.empty_like(fi)
    txt_n = torch.empty_like(ft)
    ni = torch.empty(B, device=dev)
    nt = torch.empty(C, device=dev)
    ops.l2norm_rows(fi, img_n, ni)
    ops.l2norm_rows(ft, txt_n, nt)
    probs = torch.empty(B, C, device=dev)
    dlog = torch.empty(B, C, device=dev)
    loss = torch.zeros(1, device=dev)
    ops.clip_head(img_n, txt_n, ls, y, probs, dlog, loss)
    assert rel(probs, probs_ref) < 1e-5
    assert abs(loss.item() - loss_ref.item()) < 1e-5
    di = torch.empty_like(fi)
    dt = torch.empty_like(ft)
    ops.head_feat_grad(dlog, C, 1, txt_n, img_n, ni, ls, di)
    ops.head_feat_grad(dlog, 1, C, img_n, txt_n, nt, ls, dt)
    assert rel(di, fir.grad) < 1e-4
    assert rel(dt, ftr.grad) < 1e-4
    # module-path kernels: logits/probs and softmax backward
    lg = torch.empty(B, C, device=dev)
    pr = torch.empty(B, C, device=dev)
    ops.head_logits(img_n, txt_n, ls, lg, pr)
    assert rel(lg, logits) < 1e-5 and rel(pr, probs_ref) < 1e-5
    dp = torch.randn(B, C, device=dev)
    dl = torch.empty(B, C, device=dev)
    ops.softmax_bwd_rows(pr, dp, dl)
    assert rel(dl, pr * (dp - (pr * dp).sum(-1, keepdim=True))) < 1e-5


def test_cast_weights_batch(ops, dev):
    """lc_cast_weights_bf16: several matrices (ragged shapes, with and without the transposed
    copy) in one launch, bit-equal to torch's round-to-nearest-even bf16 cast."""
    g = torch.Generator(device=dev).manual_seed(7)
    shapes = [(64, 768), (768, 64), (5, 130), (129, 3), (64, 512)]
    items = []
    for i, (n, k) in enumerate(shapes):
        W = torch.randn(n, k, device=dev, generator=g)
        out = torch.empty(n, k, device=dev, dtype=BF)
        outT = torch.empty(k, n, device=dev, dtype=BF) if i % 2 == 0 else None
        items.append((W, out, outT))
    ops.cast_weights(items)
    torch.cuda.synchronize()
    for W, out, outT in items:
        assert torch.equal(out, W.to(BF))
        if outT is not None:
            assert torch.equal(outT, W.t().to(BF))


def test_merge_weights_batch(ops, dev):
    """lc_merge_weights_bf16: LoRA merges (W + s B A, r = 1..4, with and without the transposed
    copy) and plain casts mixed in one launch, bit-equal to one lc_merge_weight per item and
    within bf16 rounding of torch fp32; more items than one launch holds (CAST_MAX)."""
    g = torch.Generator(device=dev).manual_seed(11)
    items, singles = [], []
    shapes = [(2304, 768, 4), (768, 768, 4), (4, 768, 0), (768, 4, 0), (1536, 512, 3),
              (130, 70, 1), (3, 5, 2)] * 10
    for i, (n, k, r) in enumerate(shapes):
        W = torch.randn(n, k, device=dev, generator=g)
        A = torch.randn(r, k, device=dev, generator=g) if r else None
        B = torch.randn(n, r, device=dev, generator=g) if r else None
        s = 0.5 + i / len(shapes)
        out = torch.empty(n, k, device=dev, dtype=BF)
        outT = torch.empty(k, n, device=dev, dtype=BF) if i % 3 else None
        items.append((W, A, B, s, out, outT))
        o1 = torch.empty_like(out)
        t1 = torch.empty_like(outT) if outT is not None else None
        ops.merge_weight(W, A, B, s, o1, t1)
        singles.append((o1, t1))
    assert len(items) > ops.CAST_MAX
    ops.merge_weights(items)
    torch.cuda.synchronize()
    for (W, A, B, s, out, outT), (o1, t1) in zip(items, singles):
        assert torch.equal(out, o1)
        ref = W + (s * B @ A if A is not None else 0)
        assert (out.float() - ref).abs().max() <= 2 ** -7 * ref.abs().max() + 1e-6
        if outT is not None:
            assert torch.equal(outT, t1) and torch.equal(outT, out.t())


@pytest.mark.parametrize("M,K,N", [(50432, 768, 2304), (3000 + 17, 768, 768), (770, 512, 1536),
                                   (31, 512, 512), (1, 768, 768)])
def test_lora_grad_one_pass(ops, dev, M, K, N):
    """The one-pass LoRA gradient kernel (lc_lora_grad_ws) vs torch fp32 on the same bf16
    operands: dB += s dY^T (X A^T), dA += s (dY B)^T X, r = 4, accumulated into nonzero
    buffers; ragged M (row blocks of 32 with clamped tail rows), a single row, both sites'
    shapes of the image and text towers. XA and dYB are rounded to bf16 inside the kernel (the
    MFMA operand), as in the four-GEMM form: 4e-3 relative."""
    torch.manual_seed(M + N)
    r, s = 4, 0.25
    X = torch.randn(M, K, device=dev).to(BF)
    dY = (torch.randn(M, N, device=dev) * 0.1).to(BF)
    A = torch.randn(r, K, device=dev) * K ** -0.5
    B = torch.randn(N, r, device=dev) * 0.3
    a_pad = torch.zeros(64, K, device=dev, dtype=BF)
    a_pad[:r] = A.to(BF)
    bt_pad = torch.zeros(64, N, device=dev, dtype=BF)
    bt_pad[:r] = B.t().to(BF)
    dA0 = torch.randn(r, K, device=dev)
    dB0 = torch.randn(N, r, device=dev)
    dA, dB = dA0.clone(), dB0.clone()
    ops.lora_grad_1p(dY, X, a_pad, bt_pad, r, s, dA, dB)
    xa = (X.float() @ a_pad[:r].float().t()).to(BF).float()
    dyb = (dY.float() @ bt_pad[:r].float().t()).to(BF).float()
    ref_b = s * dY.float().t() @ xa
    ref_a = s * dyb.t() @ X.float()
    assert rel(dB - dB0, ref_b) < 4e-3
    assert rel(dA - dA0, ref_a) < 4e-3
    # deterministic: the same call twice gives the same bits
    dA2, dB2 = dA0.clone(), dB0.clone()
    ops.lora_grad_1p(dY, X, a_pad, bt_pad, r, s, dA2, dB2)
    assert torch.equal(dA, dA2) and torch.equal(dB, dB2)


@pytest.mark.parametrize("M,D,keep", [(50432, 768, 1.0), (3000 + 5, 768, 0.9), (770, 512, 1.0),
                                      (7, 512, 0.9)])
def test_adapter_ln_fwd_matches_separate(ops, dev, M, D, keep):
    """The fused adapter + LayerNorm forward (lc_adapter_ln_fwd) against the separate
    lc_adapter_fwd + lc_layernorm_fwd launches and against torch fp32: same dropout mask (same
    seed), x_out / mean / rstd to f32 rounding, h and the LayerNorm output to bf16 rounding
    (the down projection sums K over the waves in a different order, so a bf16 rounding of h
    can flip); ragged M and a tail block of 7 rows."""
    torch.manual_seed(M + D)
    z = torch.randn(M, D, device=dev).to(BF)
    Wd = (torch.randn(64, D, device=dev) * D ** -0.5).to(BF)
    Wu = (torch.randn(D, 64, device=dev) * 0.125).to(BF)
    bd = torch.randn(64, device=dev) * 0.1
    bu = torch.randn(D, device=dev) * 0.1
    x = torch.randn(M, D, device=dev) * 2
    gam = torch.randn(D, device=dev)
    bet = torch.randn(D, device=dev)
    seed = 12345
    xo1, h1 = torch.empty(M, D, device=dev), torch.empty(M, 64, device=dev, dtype=BF)
    y1 = torch.empty(M, D, device=dev, dtype=BF)
    m1, r1 = torch.empty(M, device=dev), torch.empty(M, device=dev)
    ops.adapter_fwd(z, Wd, bd, Wu, bu, 0.1, keep, seed, x, xo1, h1)
    ops.layernorm_fwd(xo1, gam, bet, y1, m1, r1)
    xo2, h2 = torch.empty_like(xo1), torch.empty_like(h1)
    y2, m2, r2 = torch.empty_like(y1), torch.empty_like(m1), torch.empty_like(r1)
    ops.adapter_ln_fwd(z, Wd, bd, Wu, bu, 0.1, keep, seed, x, xo2, h2, gam, bet, y2, m2, r2)
    assert rel(h2, h1) < 4e-3
    assert ((h1 == 0) != (h2 == 0)).float().mean().item() < 1e-3  # same relu / dropout zeros
    assert rel(xo2, xo1) < 1e-5
    assert rel(m2, m1) < 1e-5 and rel(r2, r1) < 1e-5
    assert rel(y2, y1) < 4e-3
    # and against a torch fp32 restatement of adapter.py:53-72 + model.py:440-441 + the LayerNorm
    # (the kernel's dropout pattern taken from its h; the up projection on its bf16 h, as the
    # MFMA operand is): h to bf16 rounding, x_out / statistics to f32 rounding, y to bf16
    pre = z.float() @ Wd.float().t() + bd
    h_ref = torch.relu(pre) * (h2 != 0) / keep
    assert rel(h2.float(), h_ref) < 4e-3
    xo_ref = x + z.float() + 0.1 * (h2.float() @ Wu.float().t() + bu)
    assert rel(xo2, xo_ref) < 1e-5
    mu = xo_ref.mean(1)
    rs = torch.rsqrt(((xo_ref - mu[:, None]) ** 2).mean(1) + 1e-5)
    assert rel(m2, mu) < 1e-5 and rel(r2, rs) < 1e-5
    y_ref = (xo_ref - mu[:, None]) * rs[:, None] * gam + bet
    assert rel(y2.float(), y_ref) < 4e-3


@pytest.mark.parametrize("n,npch,D", [(3, 196, 768), (5, 49, 512), (256, 196, 768),
                                      (2, 256, 1024)])
def test_vit_embed_ln_matches_separate(ops, dev, n, npch, D):
    """lc_vit_embed_ln (CLS / positional embedding + ln_pre + the first block's ln_1 in one
    launch) against the separate vit_assemble + two layernorm_fwd launches (x0, statistics to
    f32 rounding, y to bf16 rounding) and against torch fp32
    (model.py:759-766, 194-200; y to bf16 rounding)."""
    torch.manual_seed(n + D)
    L = npch + 1
    pe = torch.randn(n * npch, D, device=dev)
    cls = torch.randn(D, device=dev)
    pos = torch.randn(L, D, device=dev) * 0.1
    gp, bp = torch.randn(D, device=dev), torch.randn(D, device=dev)
    g1, b1 = torch.randn(D, device=dev), torch.randn(D, device=dev)
    x0 = torch.empty(n * L, D, device=dev)
    y = torch.empty(n * L, D, device=dev, dtype=BF)
    m1, r1 = torch.empty(n * L, device=dev), torch.empty(n * L, device=dev)
    ops.vit_embed_ln(pe, cls, pos, gp, bp, g1, b1, x0, y, m1, r1, n, npch)
    xa = torch.empty(n * L, D, device=dev)
    ops.vit_assemble(pe, cls, pos, xa, n, npch)
    x0s = torch.empty_like(x0)
    ops.layernorm_fwd(xa, gp, bp, x0s, None, None)
    ys = torch.empty_like(y)
    m1s, r1s = torch.empty_like(m1), torch.empty_like(r1)
    ops.layernorm_fwd(x0s, g1, b1, ys, m1s, r1s)
    assert rel(x0, x0s) < 1e-6 and rel(m1, m1s) < 1e-6 and rel(r1, r1s) < 1e-6
    assert rel(y, ys) < 1e-3
    xr = torch.cat([cls[None].expand(n, 1, D), pe.view(n, npch, D)], 1) + pos
    x0r = torch.nn.functional.layer_norm(xr, (D,), gp, bp, 1e-5).reshape(n * L, D)
    yr = torch.nn.functional.layer_norm(x0r, (D,), g1, b1, 1e-5)
    assert rel(x0, x0r) < 1e-5
    assert rel(y, yr) < 4e-3
    assert rel(m1, x0r.mean(1)) < 1e-5


# ------------------------------------------------- the image tower's half residual stream (x16)
H16 = torch.float16


@pytest.mark.parametrize("M,D,keep", [(4096 + 7, 768, 0.9), (1000, 512, 1.0), (50432, 768, 0.9),
                                      (16 * 256 * 3 + 5, 512, 0.9)])
def test_adapter_ln_fwd_x16(ops, dev, M, D, keep):
    """lc_adapter_ln_fwd_x16 (resid and x_out in IEEE half, the reference's autocast residual
    dtype) against the f32 kernel on the same half inputs: x_out is the f32 result rounded to
    half, bit for bit (the same arithmetic, then one RNE rounding); h bit-identical; the
    LayerNorm reads x_out as stored (statistics and y against torch fp32 on the half values).
    The cases run walkers over 1, 2, 4 and 13 blocks, ragged last blocks included."""
    torch.manual_seed(M + D)
    z = torch.randn(M, D, device=dev).to(BF)
    Wd = (torch.randn(64, D, device=dev) * D ** -0.5).to(BF)
    Wu = (torch.randn(D, 64, device=dev) * 0.125).to(BF)
    bd = torch.randn(64, device=dev) * 0.1
    bu = torch.randn(D, device=dev) * 0.1
    xh = (torch.randn(M, D, device=dev) * 2).to(H16)
    gam, bet = torch.randn(D, device=dev), torch.randn(D, device=dev)
    seed = 777
    xo1, h1 = torch.empty(M, D, device=dev), torch.empty(M, 64, device=dev, dtype=BF)
    y1 = torch.empty(M, D, device=dev, dtype=BF)
    m1, r1 = torch.empty(M, device=dev), torch.empty(M, device=dev)
    ops.adapter_ln_fwd(z, Wd, bd, Wu, bu, 0.1, keep, seed, xh.float(), xo1, h1, gam, bet, y1, m1, r1)
    xo2, h2 = torch.full((M, D), float("nan"), device=dev, dtype=H16), torch.empty_like(h1)
    y2, m2, r2 = torch.empty_like(y1), torch.empty_like(m1), torch.empty_like(r1)
    ops.adapter_ln_fwd(z, Wd, bd, Wu, bu, 0.1, keep, seed, xh, xo2, h2, gam, bet, y2, m2, r2)
    assert torch.equal(h2, h1)
    assert torch.equal(xo2, xo1.to(H16))
    xr = xo2.float()
    mu = xr.mean(1)
    rs = torch.rsqrt(((xr - mu[:, None]) ** 2).mean(1) + 1e-5)
    assert rel(m2, mu) < 1e-5 and rel(r2, rs) < 1e-5
    assert rel(y2.float(), (xr - mu[:, None]) * rs[:, None] * gam + bet) < 4e-3
    with pytest.raises(ValueError):  # one dtype for resid and x_out
        ops.adapter_ln_fwd(z, Wd, bd, Wu, bu, 0.1, keep, seed, xh.float(), xo2, h2, gam, bet, y2,
                           m2, r2)


@pytest.mark.parametrize("n,npch,D", [(3, 196, 768), (5, 49, 512), (256, 196, 768)])
def test_vit_embed_ln_x16(ops, dev, n, npch, D):
    """lc_vit_embed_ln_x16: x0 is the f32 kernel's x0 rounded to half, bit for bit, and the first
    ln_1 reads x0 as stored (against torch fp32 on the half x0)."""
    torch.manual_seed(n + D + 1)
    L = npch + 1
    pe = torch.randn(n * npch, D, device=dev)
    cls, pos = torch.randn(D, device=dev), torch.randn(L, D, device=dev) * 0.1
    gp, bp = torch.randn(D, device=dev), torch.randn(D, device=dev)
    g1, b1 = torch.randn(D, device=dev), torch.randn(D, device=dev)
    x0f, y = torch.empty(n * L, D, device=dev), torch.empty(n * L, D, device=dev, dtype=BF)
    m1, r1 = torch.empty(n * L, device=dev), torch.empty(n * L, device=dev)
    ops.vit_embed_ln(pe, cls, pos, gp, bp, g1, b1, x0f, y, m1, r1, n, npch)
    x0h = torch.empty(n * L, D, device=dev, dtype=H16)
    yh = torch.empty_like(y)
    m1h, r1h = torch.empty_like(m1), torch.empty_like(r1)
    ops.vit_embed_ln(pe, cls, pos, gp, bp, g1, b1, x0h, yh, m1h, r1h, n, npch)
    assert torch.equal(x0h, x0f.to(H16))
    yr = torch.nn.functional.layer_norm(x0h.float(), (D,), g1, b1, 1e-5)
    assert rel(yh.float(), yr) < 4e-3
    xr = x0h.float()
    mu = xr.mean(1)
    assert rel(m1h, mu) < 1e-5
    assert rel(r1h, torch.rsqrt(((xr - mu[:, None]) ** 2).mean(1) + 1e-5)) < 1e-5


@pytest.mark.parametrize("D", [768, 512, 64])
def test_layernorm_x16(ops, dev, D):
    """LayerNorm forward (plain and row-gathered, as ln_post) and backward reading a half x:
    equal to the f32 kernels on x.float() (the same arithmetic on the same values)."""
    torch.manual_seed(D)
    M = 3000
    xh = (torch.randn(M, D, device=dev) * 3).to(H16)
    gam, bet = torch.randn(D, device=dev), torch.randn(D, device=dev)
    idx = torch.arange(0, M, 197, device=dev, dtype=torch.int32)
    for rows, ri in ((M, None), (idx.numel(), idx)):
        yf, yh = (torch.empty(rows, D, device=dev) for _ in range(2))
        mf, rf, mh, rh = (torch.empty(rows, device=dev) for _ in range(4))
        ops.layernorm_fwd(xh.float(), gam, bet, yf, mf, rf, row_idx=ri)
        ops.layernorm_fwd(xh, gam, bet, yh, mh, rh, row_idx=ri)
        assert torch.equal(yh, yf) and torch.equal(mh, mf) and torch.equal(rh, rf)
        dy = torch.randn(rows, D, device=dev).to(BF)
        dres = torch.randn(M, D, device=dev)
        outs = []
        for x in (xh.float(), xh):
            dx = dres.clone() * 0
            dxb = torch.zeros(M, D, device=dev, dtype=BF)
            ops.layernorm_bwd(dy, x, mf, rf, gam, dx, dxb, dres=dres if ri is None else None,
                              row_idx=ri)
            outs.append((dx, dxb))
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("D", [768, 512, 64])
def test_layernorm_bwd_g16(ops, dev, D):
    """LayerNorm backward with the residual gradient in half (dres in, dx out, lc_layernorm_bwd_g16):
    dx is the f32 kernel's result (on dres.float()) rounded to half, bit for bit, and the bf16
    copy is that half value rounded to bf16."""
    torch.manual_seed(D + 5)
    M = 2000
    xh = (torch.randn(M, D, device=dev) * 3).to(H16)
    gam, bet = torch.randn(D, device=dev), torch.randn(D, device=dev)
    y, mu, rs = torch.empty(M, D, device=dev, dtype=BF), torch.empty(M, device=dev), torch.empty(M, device=dev)
    ops.layernorm_fwd(xh, gam, bet, y, mu, rs)
    dy = (torch.randn(M, D, device=dev) * 100).to(BF)
    dres = (torch.randn(M, D, device=dev) * 50).to(H16)
    dx32, dxb32 = torch.empty(M, D, device=dev), torch.empty(M, D, device=dev, dtype=BF)
    ops.layernorm_bwd(dy, xh, mu, rs, gam, dx32, dxb32, dres=dres.float())
    dx16 = torch.full((M, D), float("nan"), device=dev, dtype=H16)
    dxb16 = torch.empty_like(dxb32)
    ops.layernorm_bwd(dy, xh, mu, rs, gam, dx16, dxb16, dres=dres)
    assert torch.equal(dx16, dx32.to(H16))
    assert torch.equal(dxb16, dx16.float().to(BF))
    # without the copy (the adapter tower): the same half result
    dxn = torch.full((M, D), float("nan"), device=dev, dtype=H16)
    ops.layernorm_bwd(dy, xh, mu, rs, gam, dxn, None, dres=dres)
    assert torch.equal(dxn, dx16)
    # row-gathered, no dres (ln_post's backward into the CLS rows)
    idx = torch.arange(0, M, 197, device=dev, dtype=torch.int32)
    dl = torch.randn(idx.numel(), D, device=dev) * 10
    g32, g16 = torch.zeros(M, D, device=dev), torch.zeros(M, D, device=dev, dtype=H16)
    b32, b16 = (torch.zeros(M, D, device=dev, dtype=BF) for _ in range(2))
    ops.layernorm_bwd(dl, xh, mu[idx.long()], rs[idx.long()], gam, g32, b32, row_idx=idx)
    ops.layernorm_bwd(dl, xh, mu[idx.long()], rs[idx.long()], gam, g16, b16, row_idx=idx)
    assert torch.equal(g16, g32.to(H16))
    with pytest.raises(ValueError):  # a half gradient needs a half x
        ops.layernorm_bwd(dy, xh.float(), mu, rs, gam, dx16, dxb16, dres=dres)


def test_adapter_wgrad_unscaled(ops, dev):
    """lc_adapter_wgrad_ws_unscaled divides every weight / bias gradient by the device scale
    (a power of two: exactly the unscaled launch's result on unscaled operands)."""
    torch.manual_seed(9)
    M, D = 50432 // 8, 768
    s = 2.0 ** 13
    g = torch.randn(M, D, device=dev).to(BF)
    h = torch.randn(M, 64, device=dev).to(BF)
    z = torch.randn(M, D, device=dev).to(BF)
    dp = torch.randn(M, 64, device=dev).to(BF)
    outs = []
    for scaled in (False, True):
        bufs = [torch.zeros(D, 64, device=dev), torch.zeros(D, device=dev),
                torch.zeros(64, D, device=dev), torch.zeros(64, device=dev)]
        if scaled:
            gs = torch.full((1,), s, device=dev)
            ops.adapter_wgrad((g.float() * s).to(BF), h, z, (dp.float() * s).to(BF), 0.1, *bufs,
                              gscale=gs)
        else:
            ops.adapter_wgrad(g, h, z, dp, 0.1, *bufs)
        outs.append(bufs)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("D,M", [(768, 50432), (768, 3152), (512, 2013), (768, 394), (768, 31)])
def test_adapter_g16(ops, dev, D, M):
    """The adapter backward launches on the half residual gradient itself (no bf16 copy):
    lc_adapter_bwd_g16 against torch fp32 of the f16 product it forms (gout exact, Wu cast to
    half; dz = gout + dpre Wd), dz and dpre-only forms; lc_adapter_wgrad_ws_unscaled_g16 bit for
    bit what the bf16-copy launch gives (the copy lc_layernorm_bwd_g16 writes: bf16 of the half
    value). Includes gradients in half's subnormal range and row counts below one walker block
    (adapter.py:59-72 autograd)."""
    torch.manual_seed(D + M)
    H16 = torch.float16
    g32 = torch.randn(M, D, device=dev) * 2.0 ** torch.randint(-22, 4, (M, 1), device=dev)
    g16 = g32.to(H16)
    gb = g16.float().to(BF)  # the copy: norm.hip rounds the stored half value to bf16
    h = torch.relu(torch.randn(M, 64, device=dev)).to(BF)
    z = torch.randn(M, D, device=dev).to(BF)
    Wu = (torch.randn(D, 64, device=dev) * 0.125).to(BF)
    Wd = (torch.randn(64, D, device=dev) * D ** -0.5).to(BF)
    WuT, WdT = Wu.t().contiguous(), Wd.t().contiguous()
    gs = torch.full((1,), 2.0 ** 12, device=dev)
    dpre = torch.full((M, 64), 7.0, device=dev, dtype=BF)
    dz = torch.full((M, D), 7.0, device=dev, dtype=BF)
    ops.adapter_bwd(g16, h, WuT, WdT, 0.1, 0.9, dpre, dz)
    dpre1 = torch.full((M, 64), 7.0, device=dev, dtype=BF)
    ops.adapter_bwd(g16, h, WuT, WdT, 0.1, 0.9, dpre1, None)
    torch.cuda.synchronize()
    dh = 0.1 * g16.float() @ Wu.half().float()
    dpr = torch.where(h.float() > 0, dh / 0.9, torch.zeros_like(dh))
    assert rel(dpre, dpr) < 4e-3
    assert torch.equal(dpre1, dpre)
    assert rel(dz, g16.float() + dpre.float() @ Wd.float()) < 4e-3
    res = {}
    for name, g in (("copy", gb), ("g16", g16)):
        bufs = [torch.zeros(D, 64, device=dev), torch.zeros(D, device=dev),
                torch.zeros(64, D, device=dev), torch.zeros(64, device=dev)]
        ops.adapter_wgrad(g, h, z, dpre, 0.1, *bufs, gscale=gs)
        torch.cuda.synchronize()
        res[name] = bufs
    for a, b in zip(res["copy"], res["g16"]):
        assert torch.equal(a, b)
    assert rel(res["g16"][0], 0.1 * gb.float().t() @ h.float() / 2.0 ** 12) < 1e-4
    with pytest.raises(TypeError):  # a half gout beside half partners has no such form
        ops.adapter_wgrad(g16, h.half(), z.half(), dpre.half(), 0.1, *bufs, gscale=gs)


@pytest.mark.parametrize("K,N", [(768, 2304), (768, 768)])
def test_lora_grad_unscaled(ops, dev, K, N):
    """lc_lora_grad_ws_unscaled (the LoRA tower's half residual gradient) divides the summed
    gradients by the device scale before the scaling and the +=: a power of two, so exactly the
    unscaled launch's result on unscaled operands (config 4's 25 216 rows, r = 4)."""
    torch.manual_seed(K + N)
    M, r, s = 25216, 4, 2.0 ** 12
    dY = (torch.randn(M, N, device=dev) * 1e-3).to(BF)
    X = torch.randn(M, K, device=dev).to(BF)
    a_pad = torch.zeros(16, K, device=dev, dtype=BF)
    bt_pad = torch.zeros(16, N, device=dev, dtype=BF)
    a_pad[:r] = torch.randn(r, K, device=dev).to(BF)
    bt_pad[:r] = torch.randn(r, N, device=dev).to(BF)
    dA0, dB0 = torch.randn(r, K, device=dev), torch.randn(N, r, device=dev)
    outs = []
    for scaled in (False, True):
        dA, dB = dA0.clone(), dB0.clone()
        if scaled:
            ops.lora_grad_1p((dY.float() * s).to(BF), X, a_pad, bt_pad, r, 0.25, dA, dB,
                             gscale=torch.full((1,), s, device=dev))
        else:
            ops.lora_grad_1p(dY, X, a_pad, bt_pad, r, 0.25, dA, dB)
        outs.append((dA, dB))
    assert not torch.equal(outs[0][0], dA0)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 8, 11])
def test_gemm_resid16(ops, dev, tile):
    """EPI_RESID16 (out0 half = aux_half + A B^T + bias: the LoRA / vanilla towers' residual add
    in the half residual stream) on every tile kernel: bit-exact on small integers (every value
    below 2^11, so exact in half), ragged M."""
    from lcclip import _lib
    lib = _lib.load()
    M, N, K = 4096 + 197, 768, 128
    g = torch.Generator(device=dev).manual_seed(tile + 40)
    A = torch.randint(-3, 4, (M, K), device=dev, generator=g).to(BF)
    B = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(BF)
    bias = torch.randint(-8, 9, (N,), device=dev, generator=g).float()
    aux = torch.randint(-500, 500, (M, N), device=dev, generator=g).to(H16)
    out = torch.full((M, N), float("nan"), device=dev, dtype=H16)
    try:
        assert lib.lc_gemm_set_tile(tile) == 0
        ops.gemm_nt(A, B, ops.EPI_RESID16, out, bias=bias, aux=aux)
    finally:
        lib.lc_gemm_set_tile(0)
    ref = A.float() @ B.float().t() + bias + aux.float()
    assert torch.equal(out, ref.to(H16))
    with pytest.raises(TypeError):
        ops.gemm_nt(A, B, ops.EPI_RESID16, out.float(), bias=bias, aux=aux)
