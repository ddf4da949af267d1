"""Phase timeline of the phase-interleaved GEMM (gemm8_kernel) from its s_memtime stamps (dev
tool). Needs the trace build:
    make -C lifelong-clip_amd/csrc TRACE=1 OBJDIR=build_trace OUT=../../exp_so/liblcclip_trace.so
    LCLIB=exp_so/liblcclip_trace.so N=768 K=3072 [FP8=1] [WG=100] python tools/g8_trace.py
Prints, per phase of the k-tile (quadrant), the median MFMA-part length (barrier exit -> MFMAs
issued), the barrier wait after it, and the LOAD-part length (the other half of the interval);
the prologue (kernel start -> loop), the loop and the epilogue, in shader cycles."""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

lib = _lib.load(os.path.join(ROOT, os.environ["LCLIB"]))
M = int(os.environ.get("M", 50432))
N, K = int(os.environ.get("N", 768)), int(os.environ.get("K", 3072))
EPI = int(os.environ.get("EPI", 0))
FP8 = os.environ.get("FP8") == "1"
WG = int(os.environ.get("WG", 0))
TN = 640
dev = torch.device("cuda:0")
lib.lc_gemm_set_tile(8)
lib.lc_gemm_set_debug.argtypes = [ctypes.c_void_p]
A = torch.randn(M, K, device=dev).to(torch.bfloat16)
B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
bias = torch.randn(N, device=dev)
o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
o1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
kw = dict(out1=o1, bias=bias) if EPI == ops.EPI_GELU_D else (dict(aux=o1) if EPI == ops.EPI_MUL else {})
if FP8:
    Aq, Bq = ops.quant_fp8(A), ops.quant_fp8(B)
    run = lambda: ops.gemm_nt_fp8(Aq, Bq, EPI, o, **kw)  # noqa: E731
else:
    run = lambda: ops.gemm_nt(A, B, EPI, o, **kw)  # noqa: E731
for _ in range(5):
    run()
dbg = torch.zeros(1 + 2 * TN, dtype=torch.int64, device=dev)
dbg[0] = WG << 32
lib.lc_gemm_set_debug(ctypes.c_void_p(dbg.data_ptr()))
run()
torch.cuda.synchronize()
lib.lc_gemm_set_debug(None)
d = dbg.cpu().tolist()
g = [d[1:1 + TN], d[1 + TN:1 + 2 * TN]]
nt = K // (128 if FP8 else 64)
t0 = g[0][0]
for grp in (0, 1):
    s = g[grp]
    print(f"group {grp}: prologue {s[1] - s[0]} cyc, loop {s[638] - s[1]} cyc "
          f"({(s[638] - s[1]) / nt:.0f}/k-tile), epilogue {s[TN - 1] - s[638]} cyc, "
          f"start offset {s[0] - t0}")
    if s[630]:
        print(f"  split slice: slab stores {s[630] - s[638]} | ticket + flag {s[631] - s[630]} | "
              f"reduce {s[632] - s[631]} | epilogue {s[TN - 1] - s[632]}")
    for p in range(4):
        mf, bw, ld = [], [], []
        for t in range(1, nt - 1):
            b = 2 + t * 12 + p * 3
            mf.append(s[b + 1] - s[b])
            bw.append(s[b + 2] - s[b + 1])
            nxt = s[b + 3] if p < 3 else s[2 + (t + 1) * 12]
            ld.append(nxt - s[b + 2])
        print(f"  phase {p}: mfma {statistics.median(mf):6.0f}  barrier-after {statistics.median(bw):6.0f}"
              f"  load-part {statistics.median(ld):6.0f}   (mean {statistics.mean(mf):.0f}/"
              f"{statistics.mean(bw):.0f}/{statistics.mean(ld):.0f})")
