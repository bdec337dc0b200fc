"""CLIP text transformer (candle ``ClipTextTransformer``; cake wraps it in
cake-core/src/models/sd/clip.rs).  Input token ids [B, 77] -> last hidden
state after ``final_layer_norm`` [B, 77, D]; causal self-attention;
quick_gelu (CLIP ViT-L) or gelu (OpenCLIP ViT-H / bigG) MLP.
Weight names: HF ``CLIPTextModel`` (``text_model.*``).
"""
from __future__ import annotations

import torch

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
        self._fused: dict = {}

    def _qkv(self, pre: str) -> tuple[torch.Tensor, torch.Tensor]:
        """The layer's q|k|v weights and biases concatenated once (cached)."""
        key = f"{pre}.self_attn.qkv@fused"
        hit = self._fused.get(key)
        if hit is None:
            names = [f"{pre}.self_attn.{n}_proj" for n in ("q", "k", "v")]
            hit = self._fused[key] = (torch.cat([self.w[f"{n}.weight"] for n in names], 0),
                                      torch.cat([self.w[f"{n}.bias"] for n in names], 0))
        return hit

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        ids = ids.long()
        B, T = ids.shape
        x = w["text_model.embeddings.token_embedding.weight"][ids] + \
            w["text_model.embeddings.position_embedding.weight"][:T][None]
        D = cfg.embed_dim
        for i in range(cfg.num_hidden_layers):
            pre = f"text_model.encoder.layers.{i}"
            h = ops.layer_norm(x, w[f"{pre}.layer_norm1.weight"], w[f"{pre}.layer_norm1.bias"],
                               cfg.layer_norm_eps)
            # q|k|v as one GEMM; attention reads the three column slices in place
            wqkv, bqkv = self._qkv(pre)
            qkv = ops.linear(h, wqkv, bqkv)
            a = ops.attention(qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:],
                              cfg.num_attention_heads, causal=True)
            x = ops.linear(a, w[f"{pre}.self_attn.out_proj.weight"],
                           w[f"{pre}.self_attn.out_proj.bias"], resid=x)  # residual fused
            h = ops.layer_norm(x, w[f"{pre}.layer_norm2.weight"], w[f"{pre}.layer_norm2.bias"],
                               cfg.layer_norm_eps)
            act = "quick_gelu" if cfg.activation == "quick_gelu" else "gelu"
            h = ops.linear(h, w[f"{pre}.mlp.fc1.weight"], w[f"{pre}.mlp.fc1.bias"], act=act)
            x = ops.linear(h, w[f"{pre}.mlp.fc2.weight"], w[f"{pre}.mlp.fc2.bias"], resid=x)
        return ops.layer_norm(x, w["text_model.final_layer_norm.weight"],
                              w["text_model.final_layer_norm.bias"], cfg.layer_norm_eps)
