"""Block-scaled fp8 path on the MI355X (BASELINE config 5): the quantiser against the oracle's
restatement of the OCP MX e4m3 format bit for bit, and the fp8 MFMA GEMM (gemm8_kernel<., true>)
against the oracle's dequantised product.

Tolerances: quantised codes and scale bytes bit-exact; the GEMM on integer data in [-8, 8]
(every value exactly representable after scaling) bit-exact; on random data the f32 output
within 3e-5 relative-norm of the fp32 product of the oracle's dequantised operands (measured
1.0e-5: the scaled MFMA's internal sum over its 128 k is not an IEEE f32 fma chain — an fp32
CPU product of the same operands differs from the exact sum by ~1e-7); bf16-output
epilogues 4e-3."""
import pytest
import torch

from oracle import clip_oracle as o

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def ops(dev):
    from lcclip import ops as _ops
    return _ops


def gpu_scales(fm):
    """[K/128, rows_pad, 4] -> [rows, K/32] (the oracle's layout)."""
    s = fm.scales.permute(1, 0, 2).reshape(fm.scales.shape[1], -1)
    return s[:fm.rows]


def ranged(rows, K, g, dev):
    """Random data whose 32-blocks span 10^-4 .. 10^4 in magnitude, with all-zero blocks,
    exact powers of two and values that saturate after scaling."""
    x = torch.randn(rows, K, generator=g, device=dev)
    mag = 10 ** (torch.rand(rows, K // 32, 1, generator=g, device=dev) * 8 - 4)
    x = (x.view(rows, K // 32, 32) * mag).view(rows, K)
    x[0, :32] = 0
    x[1, :32] = 2.0 ** torch.arange(-10, 22, device=dev).float()
    x[2, 32:64] = 448.0 * 3
    return x


@pytest.mark.parametrize("rows,K,src", [(300, 768, "bf16"), (513, 3072, "f32"), (64, 128, "f32T")])
def test_quant_fp8_bitexact(ops, dev, rows, K, src):
    g = torch.Generator(device=dev).manual_seed(rows + K)
    x = ranged(rows, K, g, dev)
    if src == "bf16":
        x = x.to(BF)
        fm = ops.quant_fp8(x)
    elif src == "f32":
        fm = ops.quant_fp8(x)
    else:  # quantise x through its transpose view (the W^T staging of the dX weights)
        xt = x.t().contiguous()
        fm = ops.quant_fp8(xt, transpose=True)
    codes, scales, _ = o.quant_fp8(x.float().cpu())
    assert fm.scales.shape == (K // 128, (rows + 255) // 256 * 256, 4)
    assert torch.equal(gpu_scales(fm).cpu(), scales)
    assert torch.equal(fm.data.cpu(), codes)


@pytest.mark.parametrize("M,N,K", [(300, 256, 128), (4096 + 197, 768, 768), (1000, 2304, 3072),
                                   (50432 // 4, 3072, 768), (12800, 768, 3072)])
def test_gemm_fp8_exact_integers(ops, dev, M, N, K):
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = torch.randint(-8, 9, (M, K), device=dev, generator=g).float()
    B = torch.randint(-8, 9, (N, K), device=dev, generator=g).float()
    Aq, Bq = ops.quant_fp8(A), ops.quant_fp8(B)
    out = torch.full((M, N), float("nan"), device=dev)
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_F32, out)
    assert torch.equal(out, A @ B.t())


@pytest.mark.parametrize("M,N,K", [(2 * 256 + 77, 768, 768), (50432, 768, 3072),
                                   (12800, 2304, 768)])
def test_gemm_fp8_vs_oracle(ops, dev, M, N, K):
    """Random operands (the split-K tail path at M = 50 432, N = 768)."""
    g = torch.Generator(device=dev).manual_seed(M * 7 + N)
    A = torch.randn(M, K, device=dev, generator=g).to(BF)
    B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5)
    bias = torch.randn(N, device=dev, generator=g)
    Aq, Bq = ops.quant_fp8(A), ops.quant_fp8(B)
    out = torch.empty(M, N, device=dev)
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_F32, out, bias=bias)
    rows = slice(0, min(M, 4096))  # oracle product on a row slice (CPU time)
    ref = o.fp8_round(A[rows].float().cpu()) @ o.fp8_round(B.cpu()).t() + bias.cpu()
    assert rel(out[rows].cpu(), ref) < 3e-5
    # the rest of the rows against the GPU's own dequantised operands
    deqA = torch.from_numpy(o.quant_fp8(A[-4096:].float().cpu())[2].numpy()).to(dev)
    ref2 = deqA @ o.fp8_round(B.cpu()).to(dev).t() + bias
    assert rel(out[-4096:], ref2) < 3e-5


def test_gemm_fp8_epilogues(ops, dev):
    M, N, K = 4096 + 131, 3072, 768
    g = torch.Generator(device=dev).manual_seed(11)
    A = torch.randn(M, K, device=dev, generator=g)
    B = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
    bias = torch.randn(N, device=dev, generator=g)
    Aq, Bq = ops.quant_fp8(A), ops.quant_fp8(B)
    ref = (o.fp8_round(A.cpu()) @ o.fp8_round(B.cpu()).t()).to(dev)
    o16 = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_BF16, o16, bias=bias)
    assert rel(o16, ref + bias) < 4e-3
    res = torch.randn(M, N, device=dev, generator=g)
    o32 = torch.empty(M, N, device=dev)
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_RESID, o32, bias=bias, aux=res)
    assert rel(o32, ref + bias + res) < 1e-5
    gd = torch.empty(M, N, device=dev, dtype=BF)
    gl = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_GELU_D, gd, bias=bias, out1=gl)
    pre = ref + bias
    s = torch.sigmoid(1.702 * pre)
    assert rel(gl, pre * s) < 4e-3
    assert rel(gd, s * (1 + 1.702 * pre * (1 - s))) < 4e-3
    aux = torch.randn(M, N, device=dev, generator=g).to(BF)
    om = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_MUL, om, alpha=0.5, aux=aux)
    assert rel(om, 0.5 * ref * aux.float()) < 4e-3


@pytest.mark.parametrize("M,N,K", [(4096 + 197, 768, 256), (12608, 768, 3072)])
def test_gemm_fp8_resid16(ops, dev, M, N, K):
    """EPI_RESID16 on the fp8 GEMM (MaPLe's c_proj forward in the half residual stream): out0
    half = aux_half + A B^T + bias, bit-exact on small integers (|v| <= 3: exact e4m3 codes under
    any block scale, every sum below 2^11), ragged M and a split-K launch (K = 3072)."""
    g = torch.Generator(device=dev).manual_seed(M + K)
    A = torch.randint(-3, 4, (M, K), device=dev, generator=g).float()
    B = torch.randint(-1, 2, (N, K), device=dev, generator=g).float()
    bias = torch.randint(-8, 9, (N,), device=dev, generator=g).float()
    aux = torch.randint(-500, 500, (M, N), device=dev, generator=g).to(torch.float16)
    out = torch.full((M, N), float("nan"), device=dev, dtype=torch.float16)
    ops.gemm_nt_fp8(ops.quant_fp8(A), ops.quant_fp8(B), ops.EPI_RESID16, out, bias=bias, aux=aux)
    ref = A @ B.t() + bias + aux.float()
    assert ref.abs().max() < 2048
    assert torch.equal(out, ref.to(torch.float16))
    with pytest.raises(TypeError):
        ops.gemm_nt_fp8(ops.quant_fp8(A), ops.quant_fp8(B), ops.EPI_RESID16, out.float(),
                        bias=bias, aux=aux)


@pytest.mark.parametrize("M,N,K", [(4096 + 131, 3072, 768), (1000, 768, 3072), (12608, 3072, 768)])
def test_gemm_fp8_q8_epilogues_match_quant(ops, dev, M, N, K):
    """The fp8-output epilogues (GELU_D_Q8 / MUL_Q8: MaPLe's c_fc forward and c_proj dX) give
    the codes and scale bytes of the bf16 epilogue followed by quant_fp8, bit for bit, and the
    same bf16 QuickGELU' — on ragged M, a split-K launch (K = 3072 at few tiles) and the
    config-5 row count."""
    g = torch.Generator(device=dev).manual_seed(M + N)
    A = torch.randn(M, K, device=dev, generator=g)
    B = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
    bias = torch.randn(N, device=dev, generator=g)
    Aq, Bq = ops.quant_fp8(A), ops.quant_fp8(B)
    blocks = N // 32

    def same(q, ref):
        assert torch.equal(q.data[:M].view(torch.uint8), ref.data[:M].view(torch.uint8))
        assert torch.equal(gpu_scales(q)[:, :blocks].view(torch.uint8),
                           gpu_scales(ref)[:, :blocks].view(torch.uint8))

    gd, gl = (torch.empty(M, N, device=dev, dtype=BF) for _ in range(2))
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_GELU_D, gd, bias=bias, out1=gl)
    gd2 = torch.empty(M, N, device=dev, dtype=BF)
    q = ops.gemm_nt_fp8(Aq, Bq, ops.EPI_GELU_D_Q8, gd2, bias=bias,
                        q_out=ops.Fp8Mat(M, N, dev))
    assert torch.equal(gd2, gd)
    same(q, ops.quant_fp8(gl))
    aux = (torch.randn(M, N, device=dev, generator=g) * 3).to(BF)
    aux[:, :64] = 0  # all-zero blocks: scale byte 0, codes 0
    om = torch.empty(M, N, device=dev, dtype=BF)
    ops.gemm_nt_fp8(Aq, Bq, ops.EPI_MUL, om, alpha=0.5, aux=aux)
    q = ops.gemm_nt_fp8(Aq, Bq, ops.EPI_MUL_Q8, None, alpha=0.5, aux=aux,
                        q_out=ops.Fp8Mat(M, N, dev))
    same(q, ops.quant_fp8(om))


@pytest.mark.parametrize("xdt", [torch.float32, torch.float16], ids=["x32", "x16"])
@pytest.mark.parametrize("rows,D", [(12608, 768), (300, 1024), (77, 256)])
def test_layernorm_fwd_fp8_matches_quant(ops, dev, rows, D, xdt):
    """LayerNorm straight into the fp8 operand format (MaPLe's ln_1 / ln_2 in fp8 mode) equals
    the bf16 LayerNorm followed by quant_fp8 bit for bit, with the same saved statistics; x f32
    or IEEE half (the half residual stream: lc_layernorm_fwd_fp8_x16)."""
    g = torch.Generator(device=dev).manual_seed(rows + D)
    x = torch.randn(rows, D, device=dev, generator=g) * 3 + 1
    x[5] = 0  # a constant row: all-zero normalised blocks when beta is 0 there
    x = x.to(xdt)
    w = torch.randn(D, device=dev, generator=g)
    b = torch.randn(D, device=dev, generator=g)
    b[:32] = 0
    y = torch.empty(rows, D, device=dev, dtype=BF)
    m1, r1 = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    ops.layernorm_fwd(x, w, b, y, m1, r1)
    ref = ops.quant_fp8(y)
    m2, r2 = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    y2 = torch.empty_like(y)
    q = ops.layernorm_fwd_fp8(x, w, b, ops.Fp8Mat(rows, D, dev), m2, r2, y=y2)
    assert torch.equal(q.data, ref.data)
    assert torch.equal(gpu_scales(q), gpu_scales(ref))
    assert torch.equal(y2, y) and torch.equal(m2, m1) and torch.equal(r2, r1)


@pytest.mark.parametrize("xdt", [torch.float32, torch.float16], ids=["x32", "x16"])
@pytest.mark.parametrize("rows,D", [(50432 // 16, 768), (301, 256), (1, 512)])
def test_layernorm_bwd_fp8_matches_quant(ops, dev, rows, D, xdt):
    """LayerNorm backward writing its result also as the fp8 operand of the next c_proj dX GEMM
    (the fp8 towers' block output gradient) equals the bf16 LayerNorm backward followed by
    quant_fp8 bit for bit, with identical f32 / bf16 outputs; with and without the residual
    gradient, and a zero output-gradient row (all-zero blocks); x f32 or IEEE half
    (lc_layernorm_bwd_fp8_x16)."""
    g = torch.Generator(device=dev).manual_seed(rows * 7 + D)
    x = (torch.randn(rows, D, device=dev, generator=g) * 2 + 0.5).to(xdt)
    w = torch.randn(D, device=dev, generator=g)
    b = torch.randn(D, device=dev, generator=g)
    y = torch.empty(rows, D, device=dev, dtype=BF)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    ops.layernorm_fwd(x, w, b, y, mean, rstd)
    dy = (torch.randn(rows, D, device=dev, generator=g) * 0.1).to(BF)
    dy[0] = 0
    for dres in (None, torch.randn(rows, D, device=dev, generator=g) * 0.01):
        if dres is not None:
            dres[0] = 0
        dx1, dxb1 = torch.empty(rows, D, device=dev), torch.empty(rows, D, device=dev, dtype=BF)
        ops.layernorm_bwd(dy, x, mean, rstd, w, dx1, dxb1, dres=dres)
        ref = ops.quant_fp8(dxb1)
        dx2, dxb2 = torch.empty_like(dx1), torch.empty_like(dxb1)
        q = ops.layernorm_bwd_fp8(dy, x, mean, rstd, w, dx2, dxb2, ops.Fp8Mat(rows, D, dev),
                                  dres=dres)
        assert torch.equal(dx2, dx1) and torch.equal(dxb2, dxb1)
        assert torch.equal(q.data, ref.data)
        assert torch.equal(gpu_scales(q), gpu_scales(ref))


@pytest.mark.parametrize("n_seq,L,H,causal", [(4, 197, 12, False), (2, 199, 12, False),
                                              (3, 77, 8, True), (2, 40, 2, False)])
def test_attn_bwd_fp8_matches_quant(ops, dev, n_seq, L, H, causal):
    """The attention backward writing dq|dk|dv as the fp8 QKV-dX operand (MaPLe's fp8 mode)
    equals attn_bwd followed by quant_fp8 bit for bit: persistent (L = 197, 199) and
    one-item-per-workgroup (L = 77 causal, 40) variants."""
    g = torch.Generator(device=dev).manual_seed(n_seq * L + H)
    D = H * 64
    M = n_seq * L
    qkv = torch.randn(M, 3 * D, device=dev, generator=g).to(BF)
    O = torch.empty(M, D, device=dev, dtype=BF)
    lse = torch.empty(n_seq * H, L, device=dev)
    ops.attn_fwd(qkv, O, lse, n_seq, L, H, causal)
    dO = torch.randn(M, D, device=dev, generator=g).to(BF)
    dqkv = torch.empty(M, 3 * D, device=dev, dtype=BF)
    ops.attn_bwd(qkv, O, dO, lse, dqkv, n_seq, L, H, causal)
    ref = ops.quant_fp8(dqkv)
    q = ops.attn_bwd_fp8(qkv, O, dO, lse, ops.Fp8Mat(M, 3 * D, dev), n_seq, L, H, causal)
    assert torch.equal(q.data, ref.data)
    assert torch.equal(gpu_scales(q), gpu_scales(ref))


def test_lora_fp8_weights_requantised_after_step(dev, ops):
    """LoRA + precision='fp8': the fused AdamW writes the LoRA parameters through the C ABI (no
    torch version bump), so after an optimizer step the re-merged QKV weight must be quantised
    again — the staged fp8 image equals quant_fp8 of the current bf16 merge, not of the old one
    (the fp8 key used to stay equal across the re-merge)."""
    from lcclip import OnlineTrainer
    from lcclip.adapter_clip import AdapterCLIP
    cfg = o.TINY_MAPLE8  # vision width 256: the fp8 tiles cover it
    sd = o.synthetic_state_dict(cfg, "lora", "both", seed=17)
    w = AdapterCLIP.from_state_dict(sd, "lora", "both", device=dev)
    stack = w.model.visual.transformer.engine
    stack.precision = "fp8"
    tr = OnlineTrainer(w, lr=5e-2)
    img = o.synthetic_images(4, cfg.image_resolution, seed=3).to(dev)
    tok = o.synthetic_tokens(3, 77, seed=3, vocab=cfg.vocab_size).to(dev)
    y = torch.tensor([0, 1, 2, 1], device=dev)
    tr.step(img, y, tok)
    st = stack.staged[0]
    before = st.q["wqkv"].data.clone()
    tr.step(img, y, tok)  # the second step's forward stages the weights AdamW moved in step 1
    torch.cuda.synchronize()
    want = ops.quant_fp8(st.wqkv)
    assert torch.equal(st.q["wqkv"].data, want.data)
    assert torch.equal(st.q["wqkv"].scales, want.scales)
    assert not torch.equal(before, want.data), "the LoRA update did not move the merged weight"


def test_fp8_keeps_non_finite(ops, dev):
    """A NaN or an infinity in a 32-block is not laundered into finite codes: the
    block gets the MX NaN scale byte 0xFF and the e4m3fn NaN code 0x7F, finite blocks are
    unchanged, and the fp8 GEMM / the MUL_Q8 epilogue carry the non-finite value on to their
    outputs (the trainer's non-finite check then skips the update)."""
    M, N, K = 300, 256, 256
    g = torch.Generator(device=dev).manual_seed(5)
    A = torch.randn(M, K, device=dev, generator=g)
    Ab = A.clone()
    Ab[3, 40] = float("nan")   # row 3, block 1
    Ab[7, 200] = float("inf")  # row 7, block 6
    Ab[9, 0] = -float("inf")   # row 9, block 0
    q, ref = ops.quant_fp8(Ab), ops.quant_fp8(A)
    s, sref = gpu_scales(q).view(torch.uint8), gpu_scales(ref).view(torch.uint8)
    bad = {(3, 1), (7, 6), (9, 0)}
    for r, b in bad:
        assert s[r, b].item() == 0xFF
        assert (q.data[r, 32 * b:32 * b + 32].view(torch.uint8) & 0x7F == 0x7F).all()
    keep = torch.ones_like(s, dtype=torch.bool)
    for r, b in bad:
        keep[r, b] = False
    assert torch.equal(s[keep], sref[keep])
    B = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
    out = torch.empty(M, N, device=dev)
    ops.gemm_nt_fp8(q, ops.quant_fp8(B), ops.EPI_F32, out)
    assert not torch.isfinite(out[[3, 7, 9]]).any(dim=1).any()
    assert torch.isfinite(out[[0, 1, 2, 4, 5, 6, 8]]).all()
    aux = torch.randn(M, N, device=dev, generator=g).to(BF)
    aux[11, 70] = float("nan")
    qo = ops.gemm_nt_fp8(ops.quant_fp8(A), ops.quant_fp8(B), ops.EPI_MUL_Q8, None, aux=aux,
                         q_out=ops.Fp8Mat(M, N, dev))
    assert gpu_scales(qo).view(torch.uint8)[11, 2].item() == 0xFF
    assert gpu_scales(qo).view(torch.uint8)[12, 2].item() != 0xFF
