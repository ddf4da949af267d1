"""Skinny GEMM microbenchmark (dev tool): the adapter down-projection shape M x 64 x 768 and the
up/add shape M x 768 x 64 through lc_gemm_nt (EPI_BF16), HIP-event timing, bytes / time.
  TILES=0,4,8 runs each listed lc_gemm_set_tile variant (0 = the selector)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
M = 50432
lib = _lib.load()
for tile in [int(t) for t in os.environ.get("TILES", "0").split(",")]:
  lib.lc_gemm_set_tile(tile)
  for N, K in ((64, 768), (768, 64)):
      A = torch.randn(M, K, device=dev).to(torch.bfloat16)
      B = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16)
      o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
      for _ in range(3):
          ops.gemm_nt(A, B, ops.EPI_BF16, o)
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      e0.record()
      for _ in range(20):
          ops.gemm_nt(A, B, ops.EPI_BF16, o)
      e1.record()
      torch.cuda.synchronize()
      us = e0.elapsed_time(e1) / 20 * 1e3
      nb = (M * K + N * K + M * N) * 2
      print(f"tile={tile} N={N:4d} K={K:4d}: {us:7.1f} us {nb / us / 1e6:5.2f} TB/s", flush=True)
lib.lc_gemm_set_tile(0)
