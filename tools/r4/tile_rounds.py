"""Per-tile time of one-round GEMM launches vs the number of busy CUs (N = 256: one column tile,
tiles = M / 256): does a tile run faster when fewer CUs are busy (clock / memory contention)?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda:0")
K = int(os.environ.get("K", 3072))
res = {}
A = torch.randn(256 * 256, K, device=dev).to(torch.bfloat16)
B = (torch.randn(256, K, device=dev) * 0.03).to(torch.bfloat16)
o = torch.empty(256 * 256, 256, device=dev, dtype=torch.bfloat16)
for rnd in range(3):
    for tiles in (64, 128, 197, 224, 256):
        M = tiles * 256
        for v in ("8", "7", "hb"):
            a, out = A[:M], o[:M]
            if v == "hb":
                f = lambda: torch.matmul(a, B.t(), out=out)  # noqa: E731
            else:
                lib.lc_gemm_set_tile(int(v))
                f = lambda: ops.gemm_nt(a, B, ops.EPI_BF16, out)  # noqa: E731
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault((tiles, v), []).append(e0.elapsed_time(e1) / 20 * 1e3)
lib.lc_gemm_set_tile(0)
for tiles in (64, 128, 197, 224, 256):
    print(f"tiles {tiles:3d} K={K}: " + " | ".join(
        f"v{v} {min(res[(tiles, v)]):6.1f} us" for v in ("8", "7", "hb")), flush=True)
