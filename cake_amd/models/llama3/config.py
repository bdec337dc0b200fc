"""Llama-3 configuration.

Parses the HF ``config.json`` fields the reference reads
(cake-core/src/models/llama3/config.rs:12-58): hidden_size, intermediate_size,
vocab_size, num_hidden_layers, num_attention_heads, num_key_value_heads
(default = num_attention_heads), rms_norm_eps, rope_theta (default 1e4),
bos/eos_token_id.  Differences: ``eos_token_id`` may be a
scalar *or* a list (Llama-3.1 configs), and ``rope_scaling`` of type "llama3" is
honoured instead of ignored.  ``MAX_SEQ_LEN`` defaults to the reference's 4096
(config.rs:5-6) and is overridable with ``--max-seq-len``.
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field
from pathlib import Path

MAX_SEQ_LEN = 4096


@dataclass
class LlamaConfig:
    hidden_size: int
    intermediate_size: int
    vocab_size: int
    num_hidden_layers: int
    num_attention_heads: int
    num_key_value_heads: int
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    bos_token_id: int | None = None
    eos_token_id: list[int] = field(default_factory=list)
    rope_scaling: dict | None = None
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    @property
    def n_rep(self) -> int:
        return self.num_attention_heads // self.num_key_value_heads

    @classmethod
    def from_dict(cls, d: dict) -> "LlamaConfig":
        eos = d.get("eos_token_id")
        eos_list = [] if eos is None else ([int(e) for e in eos] if isinstance(eos, list) else [int(eos)])
        return cls(
            hidden_size=int(d["hidden_size"]),
            intermediate_size=int(d["intermediate_size"]),
            vocab_size=int(d["vocab_size"]),
            num_hidden_layers=int(d["num_hidden_layers"]),
            num_attention_heads=int(d["num_attention_heads"]),
            num_key_value_heads=int(d.get("num_key_value_heads") or d["num_attention_heads"]),
            rms_norm_eps=float(d.get("rms_norm_eps", 1e-5)),
            rope_theta=float(d.get("rope_theta", 10000.0)),
            bos_token_id=d.get("bos_token_id") if not isinstance(d.get("bos_token_id"), list) else d["bos_token_id"][0],
            eos_token_id=eos_list,
            rope_scaling=d.get("rope_scaling"),
            max_position_embeddings=int(d.get("max_position_embeddings", 8192)),
            tie_word_embeddings=bool(d.get("tie_word_embeddings", False)),
        )

    @classmethod
    def from_path(cls, path: str | Path) -> "LlamaConfig":
        p = Path(path)
        if p.is_dir():
            p = p / "config.json"
        return cls.from_dict(json.loads(p.read_text()))

    def to_hf_dict(self) -> dict:
        d = asdict(self)
        d["eos_token_id"] = self.eos_token_id[0] if len(self.eos_token_id) == 1 else self.eos_token_id
        d["architectures"] = ["LlamaForCausalLM"]
        d["model_type"] = "llama"
        d["hidden_act"] = "silu"
        return d

    def layer_bytes(self, itemsize: int = 2) -> int:
        H, I, hd = self.hidden_size, self.intermediate_size, self.head_dim
        nh, nkv = self.num_attention_heads, self.num_key_value_heads
        return itemsize * (H * nh * hd + 2 * H * nkv * hd + nh * hd * H + 3 * H * I + 2 * H)


# Architectures of the BASELINE configs (random-init weights of these shapes).
PRESETS: dict[str, dict] = {
    "llama3-8b": dict(hidden_size=4096, intermediate_size=14336, vocab_size=128256,
                      num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=8,
                      rms_norm_eps=1e-5, rope_theta=500000.0, bos_token_id=128000,
                      eos_token_id=128009, max_position_embeddings=8192),
    "llama3-70b": dict(hidden_size=8192, intermediate_size=28672, vocab_size=128256,
                       num_hidden_layers=80, num_attention_heads=64, num_key_value_heads=8,
                       rms_norm_eps=1e-5, rope_theta=500000.0, bos_token_id=128000,
                       eos_token_id=128009, max_position_embeddings=8192),
    # tiny shape for tests: GQA 4:1, head_dim 64
    "tiny": dict(hidden_size=256, intermediate_size=512, vocab_size=512, num_hidden_layers=2,
                 num_attention_heads=4, num_key_value_heads=1, rms_norm_eps=1e-5,
                 rope_theta=500000.0, bos_token_id=1, eos_token_id=2,
                 max_position_embeddings=1024),
    # tiny with 2 KV heads: tensor-parallel tests (TP degree must divide the KV heads)
    "tiny-kv2": dict(hidden_size=256, intermediate_size=512, vocab_size=512, num_hidden_layers=2,
                     num_attention_heads=4, num_key_value_heads=2, rms_norm_eps=1e-5,
                     rope_theta=500000.0, bos_token_id=1, eos_token_id=2,
                     max_position_embeddings=1024),
}


def preset(name: str, **overrides) -> LlamaConfig:
    d = dict(PRESETS[name])
    d.update(overrides)
    return LlamaConfig.from_dict(d)
