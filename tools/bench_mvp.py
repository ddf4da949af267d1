"""MVP-CLIP step throughput (BASELINE config 3: TinyImageNet Si-Blurry, mvp_clip, 128 images per
GPU of the 512 global batch, C = 200 classes) on one MI355X: forward_features (embed, no-grad key
query over 11 blocks as methods/mvp_clip.py:298's use_last_layer default, top-1 selection, the
prompt-tuned pass at L = 202 / 217 on the prompt layers), the masked logits, loss_fn (CE +
similarity), backward to the prompts / key / mask, AdamW. Synthetic 224x224 inputs, random-init
ViT-B/16 weights. Prints one JSON line; also the split between the query pass and the rest."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lifelong-clip_amd")]
import torch  # noqa: E402

B = int(os.environ.get("B", 128))
C = int(os.environ.get("C", 200))
STEPS = int(os.environ.get("STEPS", 10))
WARM = int(os.environ.get("WARM", 3))


def main():
    from lcclip.mvp_clip import CLIP_MVP
    from lcclip.engine import ImageTower
    ImageTower.RESID16 = os.environ.get("RESID32", "0") == "0"  # A/B: f32 residual stream
    ImageTower.FUSE_EMBED = os.environ.get("FUSE_EMBED", "1") != "0"  # A/B: the separate embed
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = CLIP_MVP(model_name="ViT-B/16", device=dev, num_classes=C, use_last_layer=False)
    m.train()
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(B, 3, 224, 224, device=dev, generator=g)
    tok = torch.zeros(C, 77, dtype=torch.long, device=dev)
    tok[:, 0] = 49406
    tok[:, 1:9] = torch.randint(256, 49405, (C, 8), device=dev, generator=g)
    tok[:, 9] = 49407
    y = torch.randint(0, C, (B,), device=dev, generator=g)
    m.text_tokens = tok
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=5e-4,
                            weight_decay=1e-5)

    def step():
        opt.zero_grad(set_to_none=True)
        logits = m(x, tok)
        loss = m.loss_fn(logits, y)
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
    # the no-grad key query alone (embed + 11 blocks + ln_post)
    vis = m.backbone.visual
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.no_grad():
        e0.record()
        for _ in range(STEPS):
            x0, n, L, first = vis.tower.embed_query(x)
            vis.tower.query(x0, n, L, vis.layers - 1, first_ln1=first)
        e1.record()
    torch.cuda.synchronize()
    q_ms = e0.elapsed_time(e1) / STEPS
    print(json.dumps({"workload": "mvp_clip ViT-B/16 prompt tuning (config 3 per-GPU shape)",
                      "per_gpu_batch": B, "classes": C, "ms_per_step": round(dt * 1e3, 3),
                      "images_per_s": round(B / dt, 1), "query_pass_ms": round(q_ms, 3),
                      "dtype": "bf16", "data": "synthetic",
                      "image_residual_dtype": "f16" if ImageTower.RESID16 else "f32"}), flush=True)


if __name__ == "__main__":
    main()
