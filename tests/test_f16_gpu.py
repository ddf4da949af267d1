"""The IEEE-half (_f16) entry points the text tower runs on (include/lc_clip.h, "IEEE-half
storage"; lc_common.h compiles every 16-bit kernel source a second time with -DLC_F16): each
against a plain torch fp32 reference of the same op on the same half-rounded inputs. Half carries
a rounding of 2^-12 relative (bf16: 2^-9), so half-output checks use a relative-norm bound of
1e-3 (bf16 tests: 4e-3); exact-integer cases catch layout bugs bit-exactly. Plus the per-call
power-of-two gradient scaling of the half text tower's backward (head.hip)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

HF = torch.float16
BF = torch.bfloat16
TOL16 = 1e-3


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def ops(dev):
    from lcclip import ops as _ops
    return _ops


# --------------------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(770, 512, 512), (770, 2048, 512), (770, 512, 2048),
                                   (7700, 1536, 512), (4096 + 197, 512, 1024)])
def test_gemm_nt_f16_exact_and_epilogues(ops, dev, M, N, K):
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = torch.randint(-3, 4, (M, K), device=dev, generator=g).to(HF)
    B = torch.randint(-3, 4, (N, K), device=dev, generator=g).to(HF)
    out = torch.empty(M, N, device=dev)
    ops.gemm_nt(A, B, ops.EPI_F32, out)
    assert torch.equal(out, A.float() @ B.float().t())
    oh = torch.empty(M, N, device=dev, dtype=HF)  # small integers: exact in half too
    ops.gemm_nt(A, B, ops.EPI_BF16, oh)
    assert torch.equal(oh.float(), A.float() @ B.float().t())
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev).to(HF)
    B = (torch.randn(N, K, device=dev) * K ** -0.5).to(HF)
    bias = torch.randn(N, device=dev)
    ref = A.float() @ B.float().t() + bias
    ops.gemm_nt(A, B, ops.EPI_BF16, oh, bias=bias)
    assert rel(oh, ref) < TOL16
    res = torch.randn(M, N, device=dev)
    ops.gemm_nt(A, B, ops.EPI_RESID, out, bias=bias, aux=res)
    assert rel(out, ref + res) < 1e-5
    gd = torch.empty(M, N, device=dev, dtype=HF)
    gl = torch.empty(M, N, device=dev, dtype=HF)
    ops.gemm_nt(A, B, ops.EPI_GELU_D, gd, bias=bias, out1=gl)
    sr = torch.sigmoid(1.702 * ref)
    assert rel(gl, ref * sr) < TOL16
    assert rel(gd, sr + 1.702 * ref * sr * (1 - sr)) < TOL16
    om = torch.empty(M, N, device=dev, dtype=HF)
    ops.gemm_nt(A, B, ops.EPI_MUL, om, alpha=0.5, aux=gd)
    assert rel(om, 0.5 * (A.float() @ B.float().t()) * gd.float()) < TOL16


def test_gemm_nt_f16_rejects_mixed_types(ops, dev):
    A = torch.zeros(128, 64, device=dev, dtype=HF)
    B = torch.zeros(64, 64, device=dev, dtype=BF)
    with pytest.raises(TypeError):
        ops.gemm_nt(A, B, ops.EPI_F32, torch.empty(128, 64, device=dev))
    with pytest.raises(TypeError):
        ops.gemm_nt(A, A[:64], ops.EPI_BF16, torch.empty(128, 64, device=dev, dtype=BF))


@pytest.mark.parametrize("M,D", [(77 * 10, 512), (77 * 100 + 13, 512)])
def test_adapter_wgrad_and_gemm_tn_f16(ops, dev, M, D):
    torch.manual_seed(5)
    gout = torch.randn(M, D, device=dev).to(HF)
    z = torch.randn(M, D, device=dev).to(HF)
    h = torch.randn(M, 64, device=dev).to(HF)
    dpre = torch.randn(M, 64, device=dev).to(HF)
    dWu = torch.full((D, 64), 2.0, device=dev)
    dbu = torch.full((D,), 2.0, device=dev)
    dWd = torch.full((64, D), 2.0, device=dev)
    dbd = torch.full((64,), 2.0, device=dev)
    ops.adapter_wgrad(gout, h, z, dpre, 0.1, dWu, dbu, dWd, dbd)
    assert rel(dWu - 2, 0.1 * gout.float().t() @ h.float()) < 1e-5
    assert rel(dbu - 2, 0.1 * gout.float().sum(0)) < 1e-5
    assert rel(dWd - 2, dpre.float().t() @ z.float()) < 1e-5
    assert rel(dbd - 2, dpre.float().sum(0)) < 1e-5
    C = torch.ones(D, 64, device=dev)
    cs = torch.ones(D, device=dev)
    ops.gemm_tn(gout, h, C, alpha=0.5, colsum=cs, colsum_scale=0.25)
    assert rel(C - 1, 0.5 * gout.float().t() @ h.float()) < 1e-5
    assert rel(cs - 1, 0.25 * gout.float().sum(0)) < 1e-5


# ---------------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("D", [512, 768])
def test_layernorm_f16(ops, dev, D):
    torch.manual_seed(2)
    R = 333
    x = torch.randn(R, D, device=dev) * 3 + 1
    w, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
    y = torch.empty(R, D, device=dev, dtype=HF)
    mean, rstd = torch.empty(R, device=dev), torch.empty(R, device=dev)
    ops.layernorm_fwd(x, w, b, y, mean, rstd)
    xr = x.clone().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xr, (D,), w, b, 1e-5)
    assert rel(y, ref) < TOL16
    dy = (torch.randn(R, D, device=dev) * 1e-2).to(HF)
    ref.backward(dy.float())
    dres = torch.randn(R, D, device=dev) * 1e-2
    dx = torch.empty(R, D, device=dev)
    dxh = torch.empty(R, D, device=dev, dtype=HF)
    ops.layernorm_bwd(dy, x, mean, rstd, w, dx, dxh, dres=dres)
    assert rel(dx, xr.grad + dres) < 1e-4
    assert rel(dxh, xr.grad + dres) < TOL16
    with pytest.raises(TypeError):  # half dy with a bf16 copy: mixed types
        ops.layernorm_bwd(dy, x, mean, rstd, w, dx, torch.empty(R, D, device=dev, dtype=BF))


# ---------------------------------------------------------------------------------- attention
@pytest.mark.parametrize("n,L,H,causal", [(10, 77, 8, True), (3, 17, 2, False),
                                          (100, 77, 8, True), (2, 197, 12, False)])
def test_attention_f16(ops, dev, n, L, H, causal):
    torch.manual_seed(3)
    D = H * 64
    qkv = (torch.randn(n * L, 3 * D, device=dev) * 1.5).to(HF)
    O = torch.empty(n * L, D, device=dev, dtype=HF)
    lse = torch.empty(n * H, L, device=dev)
    ops.attn_fwd(qkv, O, lse, n, L, H, causal)
    t = qkv.float().reshape(n, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    q, k, v = (x.clone().requires_grad_(True) for x in t)
    s = (q @ k.transpose(-1, -2)) * 0.125
    if causal:
        s = s + torch.full((L, L), float("-inf"), device=dev).triu_(1)
    ref = torch.softmax(s, -1) @ v
    assert rel(O.float().reshape(n, L, H, 64).permute(0, 2, 1, 3), ref) < 2e-3
    assert rel(lse.reshape(n, H, L), torch.logsumexp(s, -1) / math.log(2)) < 1e-4
    dO = torch.randn(n * L, D, device=dev).to(HF)
    dqkv = torch.empty(n * L, 3 * D, device=dev, dtype=HF)
    ops.attn_bwd(qkv, O, dO, lse, dqkv, n, L, H, causal)
    ref.backward(dO.float().reshape(n, L, H, 64).permute(0, 2, 1, 3))
    g = dqkv.float().reshape(n, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    for i, want in enumerate((q.grad, k.grad, v.grad)):
        assert rel(g[i], want) < 5e-3, i


# ------------------------------------------------------------------------------------ adapter
@pytest.mark.parametrize("D,M,keep", [(512, 770, 1.0), (512, 7700, 0.9), (512, 3013, 1.0)])
def test_adapter_f16(ops, dev, D, M, keep):
    torch.manual_seed(D + M)
    z = torch.randn(M, D, device=dev).to(HF)
    Wd = (torch.randn(64, D, device=dev) * D ** -0.5).to(HF)
    Wu = (torch.randn(D, 64, device=dev) * 0.125).to(HF)
    bd, bu = torch.randn(64, device=dev) * 0.1, torch.randn(D, device=dev) * 0.1
    x = torch.randn(M, D, device=dev)
    xo = torch.empty(M, D, device=dev)
    h = torch.empty(M, 64, device=dev, dtype=HF)
    ops.adapter_fwd(z, Wd, bd, Wu, bu, 0.1, keep, 1234, x, xo, h)
    pre = z.float() @ Wd.float().t() + bd
    h_ref = torch.relu(pre) * (h != 0) / keep
    assert rel(h, h_ref) < TOL16
    assert rel(xo, x + z.float() + 0.1 * (h.float() @ Wu.float().t() + bu)) < 1e-5
    # fused adapter + LayerNorm: the same x_out and h, y = LN(x_out) in half
    gam, bet = torch.randn(D, device=dev), torch.randn(D, device=dev)
    xo2 = torch.empty(M, D, device=dev)
    h2 = torch.empty(M, 64, device=dev, dtype=HF)
    y2 = torch.empty(M, D, device=dev, dtype=HF)
    m2, r2 = torch.empty(M, device=dev), torch.empty(M, device=dev)
    ops.adapter_ln_fwd(z, Wd, bd, Wu, bu, 0.1, keep, 1234, x, xo2, h2, gam, bet, y2, m2, r2)
    # the fused walker splits the down projection's K across two waves: another summation
    # order than the GEMM path, so h agrees to half rounding, not bit for bit
    assert rel(h2, h) < TOL16 and rel(xo2, xo) < 1e-5
    y_ref = torch.nn.functional.layer_norm(xo, (D,), gam, bet, 1e-5)
    assert rel(y2, y_ref) < TOL16
    # backward: dpre = (h > 0) 0.1 (g Wu) / keep, dz = g + dpre Wd
    g = (torch.randn(M, D, device=dev) * 1e-2).to(HF)
    dpre = torch.empty(M, 64, device=dev, dtype=HF)
    dz = torch.empty(M, D, device=dev, dtype=HF)
    ops.adapter_bwd(g, h, Wu.t().contiguous(), Wd.t().contiguous(), 0.1, keep, dpre, dz)
    dh = 0.1 * g.float() @ Wu.float()
    dpr = torch.where(h.float() > 0, dh / keep, torch.zeros_like(dh))
    assert rel(dpre, dpr) < TOL16
    assert rel(dz, g.float() + dpre.float() @ Wd.float()) < TOL16


# ------------------------------------------------------------------------- LoRA, weight staging
@pytest.mark.parametrize("M,K,N", [(770, 512, 1536), (770, 512, 512), (7700 + 3, 512, 1536)])
def test_lora_grad_one_pass_f16(ops, dev, M, K, N):
    torch.manual_seed(M + N)
    r = 4
    dY = (torch.randn(M, N, device=dev) * 0.1).to(HF)
    X = torch.randn(M, K, device=dev).to(HF)
    A = torch.randn(r, K, device=dev) * 0.1
    B = torch.randn(N, r, device=dev) * 0.1
    a_pad = torch.zeros(64, K, device=dev, dtype=HF)
    bt_pad = torch.zeros(64, N, device=dev, dtype=HF)
    a_pad[:r] = A.to(HF)
    bt_pad[:r] = B.t().to(HF)
    dA = torch.zeros(r, K, device=dev)
    dB = torch.zeros(N, r, device=dev)
    ops.lora_grad_1p(dY, X, a_pad, bt_pad, r, 0.25, dA, dB)
    xa = (X.float() @ a_pad[:r].float().t()).to(HF).float()
    dyb = (dY.float() @ bt_pad[:r].float().t()).to(HF).float()
    assert rel(dB, 0.25 * dY.float().t() @ xa) < 2e-3
    assert rel(dA, 0.25 * dyb.t() @ X.float()) < 2e-3


def test_weight_staging_f16(ops, dev):
    torch.manual_seed(4)
    W = torch.randn(1536, 512, device=dev)
    A = torch.randn(4, 512, device=dev)
    B = torch.randn(1536, 4, device=dev)
    out = torch.empty(1536, 512, device=dev, dtype=HF)
    outT = torch.empty(512, 1536, device=dev, dtype=HF)
    ops.merge_weight(W, A, B, 0.25, out, outT)
    ref = W + 0.25 * B @ A
    assert rel(out, ref) < TOL16 and torch.equal(outT, out.t())
    items = [(torch.randn(64, 512, device=dev), torch.empty(64, 512, device=dev, dtype=HF),
              torch.empty(512, 64, device=dev, dtype=HF)) for _ in range(3)]
    ops.cast_weights(items)
    for Wi, o_, oT in items:
        assert torch.equal(o_, Wi.to(HF)) and torch.equal(oT, Wi.t().to(HF))
    ops.merge_weights([(W, A, B, 0.25, out, outT)])
    assert rel(out, ref) < TOL16
    src = torch.randn(1000, device=dev)
    dst = torch.empty(1000, device=dev, dtype=HF)
    ops.cast_bf16(src, dst)
    assert torch.equal(dst, src.to(HF))


# ---------------------------------------------------------------------- gradient scaling (head)
def test_grad_pow2_normalize_and_unscale(ops, dev):
    x = torch.randn(10, 512, device=dev) * 3e-4
    orig = x.clone()
    s = torch.empty(1, device=dev)
    ops.grad_pow2_normalize(x, s, 10)
    sv = s.item()
    assert sv == 2.0 ** round(math.log2(sv))  # a power of two
    assert 1024 <= x.abs().max().item() < 2048
    assert torch.equal(x, orig * sv)  # exact
    y = torch.ones(10 * 512, device=dev)
    ops.add_unscaled(y, x.reshape(-1), s)
    assert torch.equal(y, 1 + orig.reshape(-1))
    z = torch.zeros(64, device=dev)
    ops.grad_pow2_normalize(z, s, 10)
    assert s.item() == 1.0 and not z.any()
    z[3] = float("inf")
    ops.grad_pow2_normalize(z, s, 10)
    assert s.item() == 1.0


# ------------------------------------------------------------------------ the half text tower
def test_text_tower_f16_vs_oracle(dev):
    """ViT-B/16's 12-layer text tower (C = 10 prompts, adapter both towers, nonzero adapter
    weights) on IEEE-half storage against the oracle whose text tower rounds to half where the
    HIP path does (rt_text=round_f16), and against fp32: the half tower is closer to fp32 than
    the bf16 one (its rounding 8x finer)."""
    from lcclip.adapter_clip import AdapterCLIP
    from oracle import clip_oracle as o
    cfg = o.VIT_B16
    sd = o.synthetic_state_dict(cfg, "adapter", "both", seed=11)
    tok = o.synthetic_tokens(10, 77, seed=1)
    with torch.no_grad():
        t32 = o.encode_text(tok, sd, cfg, "adapter", "both")
        t16 = o.encode_text(tok, sd, cfg, "adapter", "both", o.round_f16)
        tbf = o.encode_text(tok, sd, cfg, "adapter", "both", o.round_bf16)
    feats = {}
    for prec in ("fp16", "bf16"):
        w = AdapterCLIP.from_state_dict(sd, "adapter", "both", device=dev, text_precision=prec)
        with torch.no_grad():
            feats[prec] = w.model.encode_text(tok.to(dev)).float().cpu()
    assert rel(feats["fp16"], t16) < 1e-3
    assert rel(feats["fp16"], t32) < 2e-3
    assert rel(feats["bf16"], tbf) < 5e-3
    assert rel(feats["fp16"], t32) < 0.5 * rel(feats["bf16"], t32)


def test_stack_apply_f16_scaled_backward(dev):
    """the plain module path (Transformer.forward -> autograd stack_apply) of an
    IEEE-half stack runs its backward on a power-of-two-scaled incoming gradient, as the fused
    towers do (engine.ScaledGrads). So its PEFT and input gradients are exactly linear in a
    power-of-two scaling of dy (bit-exact at 2^-24, where an unscaled half backward would have
    flushed the gradients to zero), and agree with the bf16 stack's within the 16-bit budget."""
    from lcclip.adapter_clip import AdapterCLIP
    from lcclip import freeze_backbone
    from oracle import clip_oracle as o
    sd = o.synthetic_state_dict(o.TINY, "adapter", "both", seed=21)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(77, 3, o.TINY.transformer_width, device=dev, generator=g)
    dy = torch.randn(x.shape, device=dev, generator=g) * 1e-4
    res = {}
    for prec, k in (("fp16", 0), ("fp16", -24), ("bf16", 0)):
        w = AdapterCLIP.from_state_dict(sd, "adapter", "both", device=dev, text_precision=prec)
        freeze_backbone(w)
        w.train()
        for m in w.modules():
            if m.__class__.__name__ == "Adapter":
                m.dropout = 0.0
        xi = x.clone().requires_grad_(True)
        y = w.model.transformer(xi)
        (y * (dy * 2.0 ** k)).sum().backward()
        peft = [p.grad * 2.0 ** -k for n, p in w.model.transformer.named_parameters()
                if p.requires_grad]
        res[(prec, k)] = (xi.grad * 2.0 ** -k, peft)
    a, b, c = res[("fp16", 0)], res[("fp16", -24)], res[("bf16", 0)]
    assert all(t.abs().sum() > 0 for t in a[1]) and a[0].abs().sum() > 0
    assert torch.equal(a[0], b[0]) and all(torch.equal(u, v) for u, v in zip(a[1], b[1]))
    assert rel(a[0], c[0]) < 2e-2
    flat = lambda r: torch.cat([t.flatten() for t in r[1]])  # noqa: E731
    assert rel(flat(a), flat(c)) < 4e-2
