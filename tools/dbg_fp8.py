"""fp8 GEMM layout probe (dev tool): plain-integer operands with hand-set E8M0 scales, to tell a
data-layout fault from a scale-mapping fault. Prints max |err| per variant."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import ops  # noqa: E402

dev = torch.device("cuda:0")
M, N, K = 256, 256, 128
g = torch.Generator(device=dev).manual_seed(0)


def mat(x, sbytes):
    """codes of x (exact small values) with scale bytes sbytes [rows, K/32]."""
    rows = x.shape[0]
    fm = ops.Fp8Mat(rows, K, dev)
    fm.data.copy_(x.to(torch.float8_e4m3fn).view(torch.uint8))
    s = sbytes.to(torch.uint8).view(rows, K // 128, 4).permute(1, 0, 2)
    fm.scales[:, :rows].copy_(s)
    return fm


def run(name, A, B, sa, sb):
    out = torch.zeros(M, N, device=dev)
    ops.gemm_nt_fp8(mat(A, sa), mat(B, sb), ops.EPI_F32, out)
    da = A * torch.exp2(sa.float() - 127).repeat_interleave(32, 1)
    db = B * torch.exp2(sb.float() - 127).repeat_interleave(32, 1)
    ref = da @ db.t()
    err = (out - ref).abs().max().item()
    print(f"{name:40s} max|err| {err:.4g}  ref max {ref.abs().max().item():.4g}", flush=True)
    return out, ref


A = torch.randint(-4, 5, (M, K), device=dev, generator=g).float()
B = torch.randint(-4, 5, (N, K), device=dev, generator=g).float()
one_a = torch.full((M, K // 32), 127, device=dev)
one_b = torch.full((N, K // 32), 127, device=dev)
run("unit scales", A, B, one_a, one_b)
run("A identity-ish rows (A = e_k)", torch.eye(M, K, device=dev), B, one_a, one_b)
sa = one_a.clone()
sa[:, 1] = 128  # block 1 of every A row x2
run("A block1 x2", A, B, sa, one_b)
sb = one_b.clone()
sb[:, 2] = 126
run("B block2 /2", A, B, one_a, sb)
sa = one_a.clone()
sa[5] = 129  # A row 5 all blocks x4
run("A row5 x4", A, B, sa, one_b)
sa = one_a.clone()
sa[:, 0] = 128
sa[:, 3] = 125
out, ref = run("A block0 x2 block3 /4", A, B, sa, one_b)
# which blocks does a lane group's scale reach? single nonzero k in A
for kk in (0, 8, 31, 32, 40, 64, 100, 127):
    Ak = torch.zeros(M, K, device=dev)
    Ak[:, kk] = 1
    sa = one_a.clone()
    sa[:, kk // 32] = 128
    o, r = run(f"A=e_{kk}, its block x2", Ak, B, sa, one_b)
    ratio = (o[0] / r[0].clamp(min=1e-9))[r[0].abs() > 0]
    print("   ratio row0:", ratio[:4].tolist())

# full map: which lane group's scale reaches each k position (scales 2^b for block b)
print("k -> log2(applied scale) (our block = k // 32)")
sa = torch.stack([torch.full((M,), 127 + b, device=dev) for b in range(4)], 1)
row = []
for kk in range(K):
    Ak = torch.zeros(M, K, device=dev)
    Ak[:, kk] = 1
    out = torch.zeros(M, N, device=dev)
    ops.gemm_nt_fp8(mat(Ak, sa), mat(B, one_b), ops.EPI_F32, out)
    ref = B[:, kk]
    nz = ref.abs() > 0
    ratio = (out[0][nz] / ref[nz]).log2().round()
    vals = sorted(set(ratio.int().tolist()))
    row.append(vals[0] if len(vals) == 1 else tuple(vals))
for b in range(4):
    print(b, row[32 * b:32 * b + 32])
