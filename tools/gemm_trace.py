"""Diagnostic: segment timestamps of the ping-pong GEMM (block 0, waves 0 and 4).
Needs a trace build: make -C lifelong-clip_amd/csrc TRACE=1 (the stamps are compiled out otherwise)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

lib = _lib.load()
M, N, K = 50432, int(os.environ.get("N", 768)), int(os.environ.get("K", 3072))
dev = torch.device("cuda:0")
lib.lc_gemm_set_tile(6)
dbg = torch.zeros(512, dtype=torch.int64, device=dev)
lib.lc_gemm_set_debug.argtypes = [ctypes.c_void_p]
A = torch.randn(M, K, device=dev).to(torch.bfloat16)
B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    ops.gemm_nt(A, B, 0, o)
lib.lc_gemm_set_debug(ctypes.c_void_p(dbg.data_ptr()))
ops.gemm_nt(A, B, 0, o)
torch.cuda.synchronize()
lib.lc_gemm_set_debug(None)
d = dbg.cpu().tolist()
t0 = min(x for x in d if x > 0)
for h in range(12):
    g0 = [d[4 * h + k] - t0 for k in range(4)]
    g1 = [d[256 + 4 * h + k] - t0 for k in range(4)]
    print(f"h={h:2d} G0 load {g0[0]:6d}->{g0[1]:6d} bar->{g0[2]:6d} comp->{g0[3]:6d} | "
          f"G1 load {g1[0]:6d}->{g1[1]:6d} bar->{g1[2]:6d} comp->{g1[3]:6d}")
steps = [d[4 * h + 4] - d[4 * h] for h in range(2, 20)]
print("G0 cycles per half (steady state):", steps)
print("G0 compute seg:", [d[4 * h + 3] - d[4 * h + 2] for h in range(2, 12)])
print("G0 load seg (to reads done):", [d[4 * h + 1] - d[4 * h] for h in range(2, 12)])
print("G0 wait+barrier:", [d[4 * h + 2] - d[4 * h + 1] for h in range(2, 12)])
