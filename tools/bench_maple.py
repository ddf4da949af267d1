"""MaPLe step throughput (BASELINE config 5 model, n_ctx 3, depth 3) on one MI355X: both towers
fwd + bwd to the prompt learner (the text tower is trained through its prompts, so it is not
cached), CE on the logits, AdamW. scripts/maple.sh:26-31 uses batch 64; C = 100 classes.
Synthetic 224x224 inputs, random-init ViT-B/16 weights. PREC=bf16|fp8|both (default both: the
image tower's frozen QKV / c_fc / c_proj GEMMs in bf16 or on the block-scaled fp8 MFMA, as
BASELINE config 5 names). Prints one JSON line per precision."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

B = int(os.environ.get("B", 64))
C = int(os.environ.get("C", 100))
STEPS = int(os.environ.get("STEPS", 10))
WARM = int(os.environ.get("WARM", 3))


def main():
    for prec in (("bf16", "fp8") if os.environ.get("PREC", "both") == "both"
                 else (os.environ["PREC"],)):
        run(prec)


def run(prec):
    from lcclip.maple import MaPLe
    from lcclip.engine import ImageTower
    ImageTower.RESID16 = os.environ.get("RESID32", "0") == "0"  # A/B: f32 residual stream
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = MaPLe("ViT-B/16", n_ctx=3, device=dev, precision=prec)
    m.overlap_text = os.environ.get("OVERLAP", "1") != "0"  # text tower on its own stream
    m.learner_on_side = os.environ.get("LEARNER_SIDE", "1") != "0"  # prompt learner there too
    m.train()
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(B, 3, 224, 224, device=dev, generator=g)
    tok = torch.zeros(C, 77, dtype=torch.long, device=dev)
    tok[:, 0] = 49406
    tok[:, 1:12] = torch.randint(256, 49405, (C, 11), device=dev, generator=g)
    tok[:, 12] = 49407
    y = torch.randint(0, C, (B,), device=dev, generator=g)
    m.set_tokenized_prompts(tok)
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=5e-4,
                            weight_decay=1e-5)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(WARM):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / STEPS
    print(json.dumps({"workload": "maple ViT-B/16 multi-modal prompts (config 5 model)",
                      "batch": B, "classes": C, "overlap_text": m.overlap_text, "ms_per_step": round(dt * 1e3, 3),
                      "images_per_s": round(B / dt, 1),
                      "dtype": "fp8 e4m3 (image QKV/c_fc/c_proj fwd+dX), bf16 elsewhere"
                      if prec == "fp8" else "bf16",
                      "data": "synthetic",
                      "image_residual_dtype": "f16" if ImageTower.RESID16 else "f32"}), flush=True)


if __name__ == "__main__":
    main()
