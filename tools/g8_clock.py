"""In-kernel clock of the phase-interleaved GEMM (gemm8_kernel) on the step's shapes (dev tool,
MI355X_MICROARCH.md 'DVFS give-back' item 6). Needs the clock build:
    bash tools/build_ab.sh WT clock -DLC_GEMM_CLOCK
    LCLIB=lifelong-clip_amd/lcclip/ab/clock.so python tools/g8_clock.py
Per shape, after >= 2 s of back-to-back launches on random data (ZERO=1: zero-filled operands),
one launch records per workgroup the shader-clock (s_memtime) and 100 MHz (s_memrealtime) cycles
around its tile. Prints the wall time and TF/s (HIP events over 50 launches), the median in-kernel
clock, and the decomposition
    frac = (clock / 2.4 GHz) x cycle_eff x slot_occ x span/wall
cycle_eff = MFMA cycles the tile needs (2MNK / 4096 flop per CU-cycle, 8192 for FP8=1) / the shader cycles the
workgroups took; slot_occ = workgroup time / (256 CUs x the grid's real-time span)."""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

lib = _lib.load(os.path.join(ROOT, os.environ["LCLIB"]))
M = int(os.environ.get("M", 50432))
ZERO = os.environ.get("ZERO") == "1"
FP8 = os.environ.get("FP8") == "1"  # the block-scaled fp8 form (MaPLe's image tower)
SHAPES = [  # (name, N, K, epi) — the bf16 step's gemm8 launches
    ("qkv_fwd", 2304, 768, ops.EPI_BF16), ("out_fwd", 768, 768, ops.EPI_BF16),
    ("fc1_fwd", 3072, 768, ops.EPI_GELU_D), ("fc2_fwd", 768, 3072, ops.EPI_RESID),
    ("fc2_dx", 3072, 768, ops.EPI_MUL), ("fc1_dx", 768, 3072, ops.EPI_BF16),
    ("qkv_dx", 768, 2304, ops.EPI_BF16),
]
PEAK, CLK_MAX = (5000.0 if FP8 else 2500.0), 2.4
FLOP_PER_CU_CYCLE = 8192 if FP8 else 4096
dev = torch.device("cuda:0")
lib.lc_gemm_set_tile(8)
lib.lc_gemm_set_debug.argtypes = [ctypes.c_void_p]
torch.manual_seed(0)
fill = (lambda *s: torch.zeros(*s, device=dev)) if ZERO else (lambda *s: torch.randn(*s, device=dev))
A = fill(M, 3072).to(torch.bfloat16)
Bw = (fill(3072, 3072) * 0.03).to(torch.bfloat16)
bias = torch.randn(3072, device=dev)
o0 = torch.empty(M * 3072, device=dev, dtype=torch.bfloat16)
o1 = torch.empty(M * 3072, device=dev, dtype=torch.bfloat16)
of = torch.empty(M, 768, device=dev)
auxf = torch.randn(M, 768, device=dev)
dbg = torch.zeros(4 * 32768, dtype=torch.int64, device=dev)
print(f"M={M} data={'zeros' if ZERO else 'random'} {'fp8' if FP8 else 'bf16'}")
for name, N, K, epi in SHAPES:
    a, b = A[:, :K].contiguous(), Bw[:N, :K].contiguous()
    out0 = o0[:M * N].view(M, N)
    kw = {}
    if epi == ops.EPI_GELU_D:
        kw = dict(out1=o1[:M * N].view(M, N), bias=bias[:N])
    elif epi == ops.EPI_MUL:
        kw = dict(aux=o1[:M * N].view(M, N))
    elif epi == ops.EPI_RESID:
        out0, kw = of, dict(aux=auxf, bias=bias[:N])
    if FP8:
        aq, bq = ops.quant_fp8(a), ops.quant_fp8(b)
        run = lambda: ops.gemm_nt_fp8(aq, bq, epi, out0, **kw)  # noqa: E731
    else:
        run = lambda: ops.gemm_nt(a, b, epi, out0, **kw)  # noqa: E731
    t_end = time.time() + 2.0
    while time.time() < t_end:
        for _ in range(20):
            run()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    wall_ms = e0.elapsed_time(e1) / 50
    for _ in range(10):  # back to the loaded state before the stamped launch
        run()
    dbg.zero_()
    lib.lc_gemm_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    run()
    lib.lc_gemm_set_debug(None)
    torch.cuda.synchronize()
    d = dbg.view(-1, 4).cpu()
    d = d[d[:, 1] > 0].double()
    if len(d) == 0:
        print(f"{name:8s} N={N:5d} K={K:5d} wall {wall_ms * 1e3:7.1f} us  (not routed to gemm8_kernel)")
        continue
    clk = statistics.median((d[:, 0] / d[:, 1] * 0.1).tolist())  # GHz
    span_s = (d[:, 3].max() - d[:, 2].min()).item() * 1e-8
    occ = d[:, 1].sum().item() * 1e-8 / (256 * span_s)
    flops = 2.0 * M * N * K
    eff = flops / FLOP_PER_CU_CYCLE / d[:, 0].sum().item()
    tf = flops / wall_ms * 1e-9
    print(f"{name:8s} N={N:5d} K={K:5d} wall {wall_ms * 1e3:7.1f} us  {tf:7.1f} TF ({tf / PEAK:.3f})  "
          f"clock {clk:.3f} GHz  cycle_eff {eff:.3f}  slot_occ {occ:.3f}  span/wall "
          f"{span_s * 1e3 / wall_ms:.3f}  WGs {len(d)}  (product {clk / CLK_MAX * eff * occ * span_s * 1e3 / wall_ms:.3f})")
