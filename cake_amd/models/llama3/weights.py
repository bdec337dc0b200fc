"""Llama-3 weight containers: load from HF safetensors or synthesise random init.

Weight names follow HF / the reference:
``model.embed_tokens.weight``, ``lm_head.weight``, ``model.norm.weight``,
``model.layers.{i}.{input_layernorm,post_attention_layernorm}.weight``,
``model.layers.{i}.self_attn.{q,k,v,o}_proj.weight``,
``model.layers.{i}.mlp.{gate,up,down}_proj.weight``; linears are [out, in].

Only the tensors a rank owns are materialised on its device (a worker never
loads the embedding or lm_head — cake-core/src/cake/worker.rs:110-125).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import torch

from .config import LlamaConfig

Getter = Callable[[str], torch.Tensor]

BLOCK_TENSORS = (
    ("ln1", "input_layernorm.weight"),
    ("wq", "self_attn.q_proj.weight"),
    ("wk", "self_attn.k_proj.weight"),
    ("wv", "self_attn.v_proj.weight"),
    ("wo", "self_attn.o_proj.weight"),
    ("ln2", "post_attention_layernorm.weight"),
    ("wg", "mlp.gate_proj.weight"),
    ("wu", "mlp.up_proj.weight"),
    ("wd", "mlp.down_proj.weight"),
)


def _materialize(t: torch.Tensor, device, dtype) -> torch.Tensor:
    """Own copy on `device` (never a view of a read-only checkpoint mapping)."""
    out = t.to(device=device, dtype=dtype)
    if out.data_ptr() == t.data_ptr():
        out = out.clone()
    return out.contiguous()


def layer_name(i: int) -> str:
    return f"model.layers.{i}"


@dataclass
class BlockWeights:
    ln1: torch.Tensor
    wq: torch.Tensor
    wk: torch.Tensor
    wv: torch.Tensor
    wo: torch.Tensor
    ln2: torch.Tensor
    wg: torch.Tensor
    wu: torch.Tensor
    wd: torch.Tensor

    def __post_init__(self):
        # q|k|v and gate|up live in one allocation each: prefill runs ONE GEMM per
        # group, and wq/wk/wv/wg/wu stay (contiguous row-slice) views for decode.
        nq, nk, ni = self.wq.shape[0], self.wk.shape[0], self.wg.shape[0]
        self.wqkv = torch.cat([self.wq, self.wk, self.wv], 0)
        self.wq, self.wk, self.wv = (self.wqkv[:nq], self.wqkv[nq:nq + nk],
                                     self.wqkv[nq + nk:])
        self.wgu = torch.cat([self.wg, self.wu], 0)
        self.wg, self.wu = self.wgu[:ni], self.wgu[ni:]

    @classmethod
    def load(cls, get: Getter, prefix: str, cfg: LlamaConfig, device, dtype) -> "BlockWeights":
        H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
        nh, nkv = cfg.num_attention_heads, cfg.num_key_value_heads
        shapes = dict(ln1=(H,), wq=(nh * hd, H), wk=(nkv * hd, H), wv=(nkv * hd, H),
                      wo=(H, nh * hd), ln2=(H,), wg=(I, H), wu=(I, H), wd=(H, I))
        out = {}
        for key, suffix in BLOCK_TENSORS:
            t = get(f"{prefix}.{suffix}")
            if tuple(t.shape) != shapes[key]:
                raise ValueError(f"{prefix}.{suffix}: shape {tuple(t.shape)} != {shapes[key]}")
            out[key] = _materialize(t, device, dtype)
        return cls(**out)

    @classmethod
    def random(cls, cfg: LlamaConfig, device, dtype, gen: torch.Generator | None = None,
               std: float = 0.02) -> "BlockWeights":
        H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
        nh, nkv = cfg.num_attention_heads, cfg.num_key_value_heads

        def lin(o, i):
            t = torch.empty((o, i), device=device, dtype=dtype)
            t.normal_(0.0, std, generator=gen)
            return t

        def norm():
            t = torch.empty((H,), device=device, dtype=dtype)
            t.normal_(1.0, 0.05, generator=gen)
            return t

        return cls(ln1=norm(), wq=lin(nh * hd, H), wk=lin(nkv * hd, H), wv=lin(nkv * hd, H),
                   wo=lin(H, nh * hd), ln2=norm(), wg=lin(I, H), wu=lin(I, H), wd=lin(H, I))

    def state_dict(self, prefix: str) -> dict[str, torch.Tensor]:
        # clones: the fused views share storage, which safetensors refuses to save
        return {f"{prefix}.{suffix}": getattr(self, key).clone() for key, suffix in BLOCK_TENSORS}


@dataclass
class HeadWeights:
    """Master-only tensors: embedding, final norm, lm_head (llama.rs:180-199)."""
    embed: torch.Tensor
    norm: torch.Tensor
    lm_head: torch.Tensor

    @classmethod
    def load(cls, get: Getter, cfg: LlamaConfig, device, dtype) -> "HeadWeights":
        emb = _materialize(get("model.embed_tokens.weight"), device, dtype)
        try:
            head = _materialize(get("lm_head.weight"), device, dtype)
        except KeyError:
            if not cfg.tie_word_embeddings:
                raise
            head = emb
        norm = _materialize(get("model.norm.weight"), device, dtype)
        return cls(embed=emb, norm=norm, lm_head=head)

    @classmethod
    def random(cls, cfg: LlamaConfig, device, dtype, gen: torch.Generator | None = None,
               std: float = 0.02) -> "HeadWeights":
        V, H = cfg.vocab_size, cfg.hidden_size
        emb = torch.empty((V, H), device=device, dtype=dtype).normal_(0.0, 1.0, generator=gen)
        head = torch.empty((V, H), device=device, dtype=dtype).normal_(0.0, std, generator=gen)
        norm = torch.empty((H,), device=device, dtype=dtype).normal_(1.0, 0.05, generator=gen)
        return cls(embed=emb, norm=norm, lm_head=head)

    def state_dict(self) -> dict[str, torch.Tensor]:
        return {"model.embed_tokens.weight": self.embed, "model.norm.weight": self.norm,
                "lm_head.weight": self.lm_head}
