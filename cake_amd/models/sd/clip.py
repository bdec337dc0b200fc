"""CLIP text transformer (candle ``ClipTextTransformer``; cake wraps it in
cake-core/src/models/sd/clip.rs).  Input token ids [B, 77] -> last hidden
state after ``final_layer_norm`` [B, 77, D]; causal self-attention;
quick_gelu (CLIP ViT-L) or gelu (OpenCLIP ViT-H / bigG) MLP.
Weight names: HF ``CLIPTextModel`` (``text_model.*``).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import ops
from .config import ClipConfig


def param_shapes(cfg: ClipConfig) -> dict[str, tuple]:
    D, I = cfg.embed_dim, cfg.intermediate_size
    p = {"text_model.embeddings.token_embedding.weight": (cfg.vocab_size, D),
         "text_model.embeddings.position_embedding.weight": (cfg.max_position_embeddings, D),
         "text_model.final_layer_norm.weight": (D,), "text_model.final_layer_norm.bias": (D,)}
    for i in range(cfg.num_hidden_layers):
        pre = f"text_model.encoder.layers.{i}"
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            p[f"{pre}.self_attn.{n}.weight"] = (D, D)
            p[f"{pre}.self_attn.{n}.bias"] = (D,)
        for n in ("layer_norm1", "layer_norm2"):
            p[f"{pre}.{n}.weight"] = (D,)
            p[f"{pre}.{n}.bias"] = (D,)
        p[f"{pre}.mlp.fc1.weight"] = (I, D)
        p[f"{pre}.mlp.fc1.bias"] = (I,)
        p[f"{pre}.mlp.fc2.weight"] = (D, I)
        p[f"{pre}.mlp.fc2.bias"] = (D,)
    return p


class ClipTextTransformer:
    def __init__(self, cfg: ClipConfig, w: dict[str, torch.Tensor]):
        self.cfg = cfg
        self.w = w

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        ids = ids.long()
        B, T = ids.shape
        x = w["text_model.embeddings.token_embedding.weight"][ids] + \
            w["text_model.embeddings.position_embedding.weight"][:T][None]
        for i in range(cfg.num_hidden_layers):
            pre = f"text_model.encoder.layers.{i}"
            h = ops.layer_norm(x, w[f"{pre}.layer_norm1.weight"], w[f"{pre}.layer_norm1.bias"],
                               cfg.layer_norm_eps)
            q = ops.linear(h, w[f"{pre}.self_attn.q_proj.weight"], w[f"{pre}.self_attn.q_proj.bias"])
            k = ops.linear(h, w[f"{pre}.self_attn.k_proj.weight"], w[f"{pre}.self_attn.k_proj.bias"])
            v = ops.linear(h, w[f"{pre}.self_attn.v_proj.weight"], w[f"{pre}.self_attn.v_proj.bias"])
            a = ops.attention(q, k, v, cfg.num_attention_heads, causal=True)
            x = x + ops.linear(a, w[f"{pre}.self_attn.out_proj.weight"],
                               w[f"{pre}.self_attn.out_proj.bias"])
            h = ops.layer_norm(x, w[f"{pre}.layer_norm2.weight"], w[f"{pre}.layer_norm2.bias"],
                               cfg.layer_norm_eps)
            h = ops.linear(h, w[f"{pre}.mlp.fc1.weight"], w[f"{pre}.mlp.fc1.bias"])
            if cfg.activation == "quick_gelu":
                h = h * torch.sigmoid(1.702 * h)
            else:
                h = F.gelu(h)
            x = x + ops.linear(h, w[f"{pre}.mlp.fc2.weight"], w[f"{pre}.mlp.fc2.bias"])
        return ops.layer_norm(x, w["text_model.final_layer_norm.weight"],
                              w["text_model.final_layer_norm.bias"], cfg.layer_norm_eps)
