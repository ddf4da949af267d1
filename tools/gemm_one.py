"""Run one lc_gemm_nt shape/variant REPS times (dev tool for PMC profiling).
env: V (tile variant), N, K, EPI (0 bf16, 3 gelu, 4 gelu_bwd), M, REPS."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

M = int(os.environ.get("M", 50432))
N, K = int(os.environ.get("N", 768)), int(os.environ.get("K", 3072))
epi = int(os.environ.get("EPI", 0))
dev = torch.device("cuda:0")
_lib.load().lc_gemm_set_tile(int(os.environ.get("V", 6)))
A = torch.randn(M, K, device=dev).to(torch.bfloat16)
B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
bias = torch.randn(N, device=dev)
o0 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
o1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
aux = torch.randn(M, N, device=dev).to(torch.bfloat16)
kw = dict(bias=bias)
if epi == 3:
    kw["out1"] = o1
if epi == 4:
    kw = dict(aux=aux)
reps = int(os.environ.get("REPS", 20))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ops.gemm_nt(A, B, epi, o0, **kw)
e0.record()
for _ in range(reps):
    ops.gemm_nt(A, B, epi, o0, **kw)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"V={os.environ.get('V')} M={M} N={N} K={K} epi={epi}: {ms*1e3:.1f} us {2*M*N*K/ms/1e9:.0f} TF/s")
