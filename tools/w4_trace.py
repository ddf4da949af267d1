"""Diagnostic (trace build, make TRACE=1): per-step stamps of the 4-wave GEMM (tile 7), wave 0
of workgroup 0: wait+barrier and issue+MFMA cycles per 32-deep step."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

lib = _lib.load(os.environ.get("LCLIB", _lib.LIB_PATH))  # a TRACE=1 build
lib.lc_gemm_set_debug.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
M, N, K = 50432, int(os.environ.get("N", 768)), int(os.environ.get("K", 3072))
A = torch.randn(M, K, device=dev).to(torch.bfloat16)
B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
lib.lc_gemm_set_tile(7)
for _ in range(3):
    ops.gemm_nt(A, B, 0, o)
dbg = torch.zeros(512, dtype=torch.int64, device=dev)
lib.lc_gemm_set_debug(ctypes.c_void_p(dbg.data_ptr()))
ops.gemm_nt(A, B, 0, o)
torch.cuda.synchronize()
lib.lc_gemm_set_debug(None)
lib.lc_gemm_set_tile(0)
d = dbg.cpu().tolist()
ns = min(K // 32, 170)
wait = [d[3 * s + 1] - d[3 * s] for s in range(ns)]
comp = [d[3 * s + 2] - d[3 * s + 1] for s in range(ns)]
print("wait+barrier:", wait[:40])
print("dma+reads+64 MFMA:", comp[:40])
print("median wait", sorted(wait)[ns // 2], "median compute", sorted(comp)[ns // 2])
