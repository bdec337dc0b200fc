"""Construct Llama-3 models for a rank: from a checkpoint directory or random init."""
from __future__ import annotations

from pathlib import Path

import torch

from .blocks import LayerStack
from .config import LlamaConfig, MAX_SEQ_LEN, preset
from .model import LlamaModel
from .weights import BlockWeights, HeadWeights, layer_name

DTYPES = {"f16": torch.float16, "bf16": torch.bfloat16, "f32": torch.float32,
          "float16": torch.float16, "bfloat16": torch.bfloat16, "float32": torch.float32}


def parse_dtype(s: str | torch.dtype) -> torch.dtype:
    if isinstance(s, torch.dtype):
        return s
    try:
        return DTYPES[s.lower()]
    except KeyError:
        raise ValueError(f"unsupported dtype {s!r} (f16, bf16, f32)") from None


def default_backend(device: torch.device, dtype: torch.dtype) -> str:
    if device.type == "cuda" and dtype in (torch.float16, torch.bfloat16):
        return "hip"
    return "torch"


def random_stack(cfg: LlamaConfig, layers: list[int], device, dtype, max_seq: int = MAX_SEQ_LEN,
                 backend: str | None = None, seed: int = 0, max_sessions: int = 8) -> LayerStack:
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    weights = {}
    for li in layers:
        gen.manual_seed(seed * 1000003 + li)
        weights[li] = BlockWeights.random(cfg, device, dtype, gen)
    return LayerStack(cfg, weights, device, dtype, max_seq, backend or default_backend(device, dtype),
                      max_sessions=max_sessions)


def random_head(cfg: LlamaConfig, device, dtype, seed: int = 0) -> HeadWeights:
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed * 7919 + 17)
    return HeadWeights.random(cfg, device, dtype, gen)


def random_model(cfg: LlamaConfig | str, device, dtype, max_seq: int = MAX_SEQ_LEN,
                 local_layers: list[int] | None = None, remote: dict | None = None,
                 backend: str | None = None, seed: int = 0) -> LlamaModel:
    if isinstance(cfg, str):
        cfg = preset(cfg)
    device = torch.device(device)
    if local_layers is None:
        local_layers = [li for li in range(cfg.num_hidden_layers) if li not in (remote or {})]
    stack = random_stack(cfg, local_layers, device, dtype, max_seq, backend, seed)
    return LlamaModel(cfg, random_head(cfg, device, dtype, seed), stack, remote)


def load_stack(model_dir: str | Path, cfg: LlamaConfig, layers: list[int], device, dtype,
               max_seq: int = MAX_SEQ_LEN, backend: str | None = None) -> LayerStack:
    from ...utils.safetensors_io import ShardedCheckpoint
    ck = ShardedCheckpoint(model_dir)
    device = torch.device(device)
    weights = {li: BlockWeights.load(ck.get, layer_name(li), cfg, device, dtype) for li in layers}
    return LayerStack(cfg, weights, device, dtype, max_seq, backend or default_backend(device, dtype))


def load_model(model_dir: str | Path, device, dtype, max_seq: int = MAX_SEQ_LEN,
               remote: dict | None = None, backend: str | None = None) -> LlamaModel:
    from ...utils.safetensors_io import ShardedCheckpoint
    cfg = LlamaConfig.from_path(model_dir)
    device = torch.device(device)
    local = [li for li in range(cfg.num_hidden_layers) if li not in (remote or {})]
    stack = load_stack(model_dir, cfg, local, device, dtype, max_seq, backend)
    ck = ShardedCheckpoint(model_dir)
    head = HeadWeights.load(ck.get, cfg, device, dtype)
    return LlamaModel(cfg, head, stack, remote)
