"""Diagnostic: prologue / main loop / epilogue of the ping-pong GEMM's workgroup 0 (s_memtime
stamps, wave 0) for the step's shapes, with the launch's wall time for scale (dev tool).
Needs a trace build: make -C lifelong-clip_amd/csrc TRACE=1."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

lib = _lib.load()
lib.lc_gemm_set_debug.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
M = 50432
for name, N, K, epi in (("qkv_fwd", 2304, 768, ops.EPI_BF16), ("fc1_fwd", 3072, 768, ops.EPI_GELU_D),
                        ("fc2_dx", 3072, 768, ops.EPI_MUL), ("fc2_fwd", 768, 3072, ops.EPI_BF16)):
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    kw = {}
    if epi == ops.EPI_GELU_D:
        kw = dict(bias=torch.randn(N, device=dev), out1=torch.empty_like(o))
    elif epi == ops.EPI_MUL:
        kw = dict(aux=torch.randn(M, N, device=dev).to(torch.bfloat16))
    for _ in range(3):
        ops.gemm_nt(A, B, epi, o, **kw)
    dbg = torch.zeros(512, dtype=torch.int64, device=dev)
    res = []
    for rep in range(5):
        dbg.zero_()
        lib.lc_gemm_set_debug(ctypes.c_void_p(dbg.data_ptr()))
        ops.gemm_nt(A, B, epi, o, **kw)
        torch.cuda.synchronize()
        lib.lc_gemm_set_debug(None)
        d = dbg.cpu().tolist()
        t0 = d[250]
        res.append((d[0] - t0, d[251] - d[0], d[252] - d[251], d[252] - t0))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.gemm_nt(A, B, epi, o, **kw)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    med = [sorted(r[i] for r in res)[2] for i in range(4)]
    print(f"{name:8s} launch {us:6.1f} us | WG0 cycles: prologue {med[0]:6d} main {med[1]:6d} "
          f"epilogue {med[2]:6d} total {med[3]:6d}", flush=True)
