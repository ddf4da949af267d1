"""GEMM microbenchmark on the ViT-B/16 step's shapes (dev tool): every lc_gemm_nt tile variant,
random bf16 operands, HIP-event timing on the launch stream, interleaved rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

M = int(os.environ.get("M", 50432))
SHAPES = [  # (name, N, K, epi)
    ("qkv_fwd", 2304, 768, ops.EPI_BF16), ("out_fwd", 768, 768, ops.EPI_BF16),
    ("fc1_fwd", 3072, 768, ops.EPI_GELU_D), ("fc2_fwd", 768, 3072, ops.EPI_BF16),
    ("fc2_dx", 3072, 768, ops.EPI_MUL), ("fc1_dx", 768, 3072, ops.EPI_BF16),
    ("out_dx", 768, 768, ops.EPI_BF16), ("qkv_dx", 768, 2304, ops.EPI_BF16),
]
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,2,3").split(",")]
dev = torch.device("cuda:0")
lib = _lib.load()
torch.manual_seed(0)
Kmax, Nmax = 3072, 3072
A = torch.randn(M, Kmax, device=dev).to(torch.bfloat16)
Bw = (torch.randn(Nmax, Kmax, device=dev) * 0.03).to(torch.bfloat16)
bias = torch.randn(Nmax, device=dev)
o0 = torch.empty(M, Nmax, device=dev, dtype=torch.bfloat16)
o1 = torch.empty(M, Nmax, device=dev, dtype=torch.bfloat16)
aux = torch.randn(M, Nmax, device=dev).to(torch.bfloat16)
res = {}
reps = int(os.environ.get("REPS", 10))
for rnd in range(3):
    for name, N, K, epi in SHAPES:
        for v in VARIANTS:
            if v in (3, 5, 6) and N % 256:
                continue
            lib.lc_gemm_set_tile(v)
            a = A[:, :K]
            b = Bw[:N, :K]
            kw = {}
            if epi in (ops.EPI_GELU, ops.EPI_GELU_D):
                kw = dict(bias=bias[:N], out1=o1[:, :N])
            elif epi in (ops.EPI_GELU_BWD, ops.EPI_MUL):
                kw = dict(aux=aux[:, :N])
            else:
                kw = dict(bias=bias[:N])
            ops.gemm_nt(a, b, epi, o0[:, :N], **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.gemm_nt(a, b, epi, o0[:, :N], **kw)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res.setdefault((name, v), []).append(ms)
lib.lc_gemm_set_tile(0)
tot = {v: 0.0 for v in VARIANTS}
for name, N, K, epi in SHAPES:
    line = f"{name:8s} N={N:5d} K={K:5d}"
    for v in VARIANTS:
        if (name, v) not in res:
            line += f" | v{v}:   -   "
            continue
        ms = min(res[(name, v)])
        tf = 2 * M * N * K / ms / 1e9
        line += f" | v{v}: {ms * 1e3:7.1f}us {tf:6.0f}TF"
    print(line, flush=True)
