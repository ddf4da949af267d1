"""Back-to-back dependent launches on one stream (dev tool): the per-kernel bubble the step pays
on its ~284 main-stream kernels. A tiny kernel (lc_cast_bf16, 64 elements) timed in a loop with
HIP events; and the same with a cross-stream event wait per launch (the side-stream syncs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import ops  # noqa: E402

dev = torch.device("cuda:0")
a = torch.randn(64, device=dev)
b = torch.empty(64, device=dev, dtype=torch.bfloat16)
side = torch.cuda.Stream(dev)


def run(n, sync):
    main = torch.cuda.current_stream(dev)
    for _ in range(n):
        ops.cast_bf16(a, b)
        if sync:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                ops.cast_bf16(a, b)
            main.wait_stream(side)


x = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
for sync in (False, True):
    run(50, sync)
    torch.cuda.synchronize()
    n = 1000
    # a long GPU prefix so that the host has queued every small launch before the GPU reaches
    # them: the events then time the GPU's per-kernel turnaround, not the host's launch rate
    for _ in range(40):
        torch.mm(x, x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run(n, sync)
    e1.record()
    torch.cuda.synchronize()
    print(f"sync={sync}: {e0.elapsed_time(e1) / n * 1e3:.2f} us per main-stream launch", flush=True)
