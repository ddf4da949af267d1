"""GEMM microbenchmark on the ViT-B/16 step's shapes (dev tool): lc_gemm_nt tile variants,
random bf16 operands, HIP-event timing on the launch stream, interleaved rounds.

  VARIANTS=1,5,5n,8,f8,s3  (5n = ping-pong without the split-K workspace, 8 = phase-interleaved
  bf16 kernel, f8 = its block-scaled fp8 form on pre-quantised operands, sK = the 8 kernel under
  lc_gemm_set_streamk(K), hb = hipBLASLt through torch.matmul)   SQUARE=1 adds 4096^3/8192^3
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

if os.environ.get("LCLIB"):  # an experimental build of the library
    _lib.load(os.path.join(ROOT, os.environ["LCLIB"]))
from lcclip._lib import call, ptr, stream_of  # noqa: E402

M = int(os.environ.get("M", 50432))
W = int(os.environ.get("W", 768))  # the tower width (512: the text tower's shapes)
SHAPES = [  # (name, M, N, K, epi)
    ("qkv_fwd", M, 3 * W, W, ops.EPI_BF16), ("out_fwd", M, W, W, ops.EPI_BF16),
    ("fc1_fwd", M, 4 * W, W, ops.EPI_GELU_D), ("fc2_fwd", M, W, 4 * W, ops.EPI_BF16),
    ("fc2_dx", M, 4 * W, W, ops.EPI_MUL), ("fc1_dx", M, W, 4 * W, ops.EPI_BF16),
    ("out_dx", M, W, W, ops.EPI_BF16), ("qkv_dx", M, W, 3 * W, ops.EPI_BF16),
]
if os.environ.get("SQUARE"):
    SHAPES += [("sq4096", 4096, 4096, 4096, ops.EPI_BF16), ("sq8192", 8192, 8192, 8192, ops.EPI_BF16)]
VARIANTS = os.environ.get("VARIANTS", "1,2,3").split(",")
dev = torch.device("cuda:0")
lib = _lib.load()
torch.manual_seed(0)
Mmax = max(s[1] for s in SHAPES)
Kmax = max(s[3] for s in SHAPES)
Nmax = max(s[2] for s in SHAPES)
A = torch.randn(Mmax, Kmax, device=dev).to(torch.bfloat16)
Bw = (torch.randn(Nmax, Kmax, device=dev) * 0.03).to(torch.bfloat16)
bias = torch.randn(Nmax, device=dev)
o0 = torch.empty(Mmax * Nmax, device=dev, dtype=torch.bfloat16)
o1 = torch.empty(Mmax * Nmax, device=dev, dtype=torch.bfloat16)
aux = torch.randn(Mmax * Nmax, device=dev).to(torch.bfloat16)


_q = {}


def launch(v, m, N, K, epi, a, b, out0, kw):
    if v == "hb":
        torch.matmul(a, b.t(), out=out0)
    elif v == "f8":
        key = (m, N, K)
        if key not in _q:
            _q[key] = (ops.quant_fp8(a), ops.quant_fp8(b))
        ops.gemm_nt_fp8(*_q[key], epi, out0, **kw)
    elif v.endswith("n"):  # no split-K workspace
        out1, ax, bs = kw.get("out1"), kw.get("aux"), kw.get("bias")
        call("lc_gemm_nt", stream_of(a), epi, m, N, K, ptr(a), a.stride(0), ptr(b), b.stride(0),
             ptr(bs), 1.0, ptr(out0), N, ptr(out1), N if out1 is not None else 0, ptr(ax),
             N if ax is not None else 0)
    else:
        ops.gemm_nt(a, b, epi, out0, **kw)


res = {}
reps = int(os.environ.get("REPS", 10))
for rnd in range(3):
    for name, m, N, K, epi in SHAPES:
        for v in VARIANTS:
            t = 8 if v in ("f8", "hb") or v.startswith("s") else int(v.rstrip("n"))
            if v.startswith("s") or hasattr(lib, "lc_gemm_set_streamk"):
                lib.lc_gemm_set_streamk(int(v[1:]) if v.startswith("s") else 0)
            if t in (3, 5, 6, 7, 8) and N % 256:
                continue
            if v != "hb" and lib.lc_gemm_set_tile(t) != 0:
                raise SystemExit(f"lc_gemm_set_tile({t}) rejected")
            a = A[:m, :K]
            b = Bw[:N, :K]
            out0 = o0[:m * N].view(m, N)
            if epi in (ops.EPI_GELU, ops.EPI_GELU_D):
                kw = dict(bias=bias[:N], out1=o1[:m * N].view(m, N))
            elif epi in (ops.EPI_GELU_BWD, ops.EPI_MUL):
                kw = dict(aux=aux[:m * N].view(m, N))
            else:
                kw = dict(bias=bias[:N])
            launch(v, m, N, K, epi, a, b, out0, kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                launch(v, m, N, K, epi, a, b, out0, kw)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res.setdefault((name, v), []).append(ms)
lib.lc_gemm_set_tile(0)
if hasattr(lib, "lc_gemm_set_streamk"):
    lib.lc_gemm_set_streamk(0)
for name, m, N, K, epi in SHAPES:
    line = f"{name:8s} M={m:6d} N={N:5d} K={K:5d}"
    for v in VARIANTS:
        if (name, v) not in res:
            line += f" | v{v}:   -   "
            continue
        ms = min(res[(name, v)])
        tf = 2 * m * N * K / ms / 1e9
        line += f" | v{v}: {ms * 1e3:7.1f}us {tf:6.0f}TF"
    print(line, flush=True)
