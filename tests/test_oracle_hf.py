"""Pin the oracle's encoder arithmetic against an independent implementation of the same
published architecture (CPU, no GPU): transformers' CLIPModel (installed here, 5.x) is a
separate implementation of OpenAI CLIP — the code the reference vendors as models/clip/model.py
(pre-LN residual blocks, QuickGELU, class + positional embeddings with ln_pre, ln_post and the
visual projection, causal text mask, EOT pooling by argmax of the token ids, L2-normalised
logits scaled by exp(logit_scale)). The reference itself cannot be executed here;
this pins oracle/clip_oracle.py's vanilla towers and logit head (encode_image, encode_text,
clip_logits; models/clip/model.py:209-245, 755-787, 938-975) element for element in fp32 on random weights, with the
state dict translated the way transformers' own OpenAI-checkpoint converter maps it. The PEFT
variants build on these blocks (adapter-at-init == vanilla and the LoRA merge identities are
pinned in tests/test_oracle.py)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import clip_oracle as o  # noqa: E402

transformers = pytest.importorskip("transformers")


def hf_config(cfg):
    from transformers import CLIPConfig
    text = dict(vocab_size=cfg.vocab_size, hidden_size=cfg.transformer_width,
                intermediate_size=4 * cfg.transformer_width,
                num_hidden_layers=cfg.transformer_layers,
                num_attention_heads=cfg.transformer_heads,
                max_position_embeddings=cfg.context_length, hidden_act="quick_gelu",
                layer_norm_eps=1e-5, eos_token_id=2, projection_dim=cfg.embed_dim)
    vision = dict(hidden_size=cfg.vision_width, intermediate_size=4 * cfg.vision_width,
                  num_hidden_layers=cfg.vision_layers, num_attention_heads=cfg.vision_heads,
                  image_size=cfg.image_resolution, patch_size=cfg.vision_patch_size,
                  hidden_act="quick_gelu", layer_norm_eps=1e-5, projection_dim=cfg.embed_dim)
    return CLIPConfig(text_config=text, vision_config=vision, projection_dim=cfg.embed_dim)


def to_hf(sd, cfg):
    """OpenAI CLIP state-dict names (the reference's / the oracle's) -> transformers' CLIPModel."""
    out = {}

    def blocks(src, dst, n, width):
        for i in range(n):
            s, d = f"{src}{i}.", f"{dst}{i}."
            w, b = sd[s + "attn.in_proj_weight"], sd[s + "attn.in_proj_bias"]
            for j, name in enumerate(("q_proj", "k_proj", "v_proj")):
                out[d + f"self_attn.{name}.weight"] = w[j * width:(j + 1) * width]
                out[d + f"self_attn.{name}.bias"] = b[j * width:(j + 1) * width]
            out[d + "self_attn.out_proj.weight"] = sd[s + "attn.out_proj.weight"]
            out[d + "self_attn.out_proj.bias"] = sd[s + "attn.out_proj.bias"]
            for a, bname in (("ln_1", "layer_norm1"), ("ln_2", "layer_norm2")):
                out[d + f"{bname}.weight"] = sd[s + f"{a}.weight"]
                out[d + f"{bname}.bias"] = sd[s + f"{a}.bias"]
            for a, bname in (("mlp.c_fc", "mlp.fc1"), ("mlp.c_proj", "mlp.fc2")):
                out[d + f"{bname}.weight"] = sd[s + f"{a}.weight"]
                out[d + f"{bname}.bias"] = sd[s + f"{a}.bias"]
    blocks("visual.transformer.resblocks.", "vision_model.encoder.layers.", cfg.vision_layers,
           cfg.vision_width)
    blocks("transformer.resblocks.", "text_model.encoder.layers.", cfg.transformer_layers,
           cfg.transformer_width)
    out["vision_model.embeddings.patch_embedding.weight"] = sd["visual.conv1.weight"]
    out["vision_model.embeddings.class_embedding"] = sd["visual.class_embedding"]
    out["vision_model.embeddings.position_embedding.weight"] = sd["visual.positional_embedding"]
    for a, b in (("visual.ln_pre", "vision_model.pre_layrnorm"),
                 ("visual.ln_post", "vision_model.post_layernorm"),
                 ("ln_final", "text_model.final_layer_norm")):
        out[b + ".weight"] = sd[a + ".weight"]
        out[b + ".bias"] = sd[a + ".bias"]
    out["visual_projection.weight"] = sd["visual.proj"].t()
    out["text_projection.weight"] = sd["text_projection"].t()
    out["text_model.embeddings.token_embedding.weight"] = sd["token_embedding.weight"]
    out["text_model.embeddings.position_embedding.weight"] = sd["positional_embedding"]
    out["logit_scale"] = sd["logit_scale"]
    return out


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("cfg,B,C", [(o.TINY, 3, 4), (o.VIT_B16, 2, 3)], ids=["tiny", "vit_b16"])
def test_oracle_vanilla_towers_match_transformers_clip(cfg, B, C):
    from transformers import CLIPModel
    sd = o.synthetic_state_dict(cfg, "vanilla", "none", seed=5)
    model = CLIPModel(hf_config(cfg)).eval()
    hf_sd = to_hf(sd, cfg)
    missing, unexpected = model.load_state_dict(hf_sd, strict=False)
    # position_ids buffers are not parameters of the reference; nothing else may be left over
    assert not unexpected and all("position_ids" in k for k in missing), (missing, unexpected)
    img = o.synthetic_images(B, cfg.image_resolution, seed=6)
    tok = o.synthetic_tokens(C, cfg.context_length, seed=7, vocab=cfg.vocab_size)
    with torch.no_grad():
        fi = o.encode_image(img, sd, cfg)
        ft = o.encode_text(tok, sd, cfg)
        logits, _, _ = o.clip_logits(fi, ft, sd["logit_scale"])
        hi = model.get_image_features(pixel_values=img)
        ht = model.get_text_features(input_ids=tok)
        hl = model(input_ids=tok, pixel_values=img).logits_per_image
    hi = getattr(hi, "pooler_output", hi)
    ht = getattr(ht, "pooler_output", ht)
    assert rel(fi, hi) < 1e-5 and rel(ft, ht) < 1e-5, (rel(fi, hi), rel(ft, ht))
    assert (logits - hl).abs().max().item() / sd["logit_scale"].exp().item() < 1e-5
