"""Feasibility probe (dev tool, GPU): does running the image tower as two half-batches on two
HIP streams beat one full-batch pass? The idea: one half's GEMM ragged rounds and HBM-bound
streaming kernels (LayerNorm, adapter, attention) overlap the other half's MFMA-bound GEMMs.

Times, on ViT-B/16 adapter (both towers' PEFT on), B images:
  full   one tower fwd + bwd over B images on the current stream (the trainer's form)
  split  two towers (same weights / engine, their own row-gradient buffers) fwd + bwd over B/2
         images each, half A on stream A, half B on stream B, enqueued A then B per phase
  serial the same two halves on one stream (the cost of halving M alone)
Weight-gradient reductions go to one shared side stream in every form.

    python tools/microbatch_probe.py [B] [REPS]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

from lcclip import AdapterCLIP, OnlineTrainer  # noqa: E402
from lcclip.engine import ImageTower  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = AdapterCLIP("ViT-B/16", peft_method="adapter", peft_encoder="both", device=dev)
    tr = OnlineTrainer(model)
    vis = model.model.visual
    full = tr.img
    halves = [ImageTower(vis, full.stack), ImageTower(vis, full.stack)]
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(B, 3, 224, 224, device=dev, generator=g)
    df = torch.randn(B, 512, device=dev, generator=g) * 1e-3
    gs = torch.cuda.Stream(device=dev)
    sa, sb = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    main = torch.cuda.current_stream(dev)
    h = B // 2

    def run_full():
        f, c = full.forward(x, save=True, training=True)
        full.backward(c, df, tr.grads, grad_stream=gs)

    def run_split(streams):
        ctxs = []
        for i, t in enumerate(halves):
            st = streams[i]
            st.wait_stream(main)
            with torch.cuda.stream(st):
                ctxs.append(t.forward(x[i * h:(i + 1) * h], save=True, training=True)[1])
        for i, t in enumerate(halves):
            with torch.cuda.stream(streams[i]):
                t.backward(ctxs[i], df[i * h:(i + 1) * h], tr.grads, grad_stream=gs)
        for st in streams:
            main.wait_stream(st)

    forms = {"full": run_full, "split": lambda: run_split((sa, sb)),
             "serial": lambda: run_split((sa, sa))}
    for fn in forms.values():  # warm-up (allocator, staging)
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in forms}
    for _ in range(3):
        for k, fn in forms.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            for _ in range(reps):
                fn()
            e1.record(main)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / reps)
    for k, v in res.items():
        print(f"{k:6s} B={B}: {min(v):7.3f} ms per tower fwd+bwd  (rounds {', '.join(f'{t:.3f}' for t in v)})",
              flush=True)


if __name__ == "__main__":
    main()
