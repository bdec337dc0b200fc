"""safetensors I/O over the native mmap reader/writer (csrc/runtime/safetensors.cpp).

Reference: cake-core/src/utils/mod.rs:32-104 (index → shard list → mmapped
VarBuilder).  Tensors are zero-copy views of the mapping until moved to the
target device, so a rank only materialises what it owns.
"""
from __future__ import annotations

from pathlib import Path

import torch

from .native import runtime

ST_DTYPES = {
    "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16, "F64": torch.float64,
    "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8,
    "U8": torch.uint8, "BOOL": torch.bool,
}
TORCH_TO_ST = {v: k for k, v in ST_DTYPES.items()}


class SafeTensors:
    def __init__(self, path: str | Path):
        self.path = str(path)
        self._f = runtime().SafeTensorsFile(self.path)
        self._buf = self._f.buffer()

    def keys(self) -> list[str]:
        return list(self._f.names())

    def metadata(self) -> dict:
        return dict(self._f.metadata())

    def __contains__(self, name: str) -> bool:
        return name in self._f

    def get(self, name: str) -> torch.Tensor:
        """Zero-copy (read-only) CPU view; `.to(device)` uploads it."""
        info = self._f.info(name)
        dt = ST_DTYPES[info["dtype"]]
        n = info["nbytes"]
        if n == 0:
            return torch.empty(info["shape"], dtype=dt)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")  # read-only mapping; we never write through it
            # frombuffer on the WHOLE mapping (not a slice) so the tensor keeps the
            # memoryview — and through it the native mapping — alive
            t = torch.frombuffer(self._buf, dtype=torch.uint8, count=n, offset=info["offset"])
        return t.view(dt).reshape(info["shape"])


class ShardedCheckpoint:
    """A HF checkpoint directory (index + shards, or a single model.safetensors)."""

    def __init__(self, model_dir: str | Path):
        self.dir = Path(model_dir)
        self.weight_map: dict[str, str] = dict(runtime().load_weight_map(str(self.dir)))
        self._files: dict[str, SafeTensors] = {}

    def get(self, name: str) -> torch.Tensor:
        try:
            fname = self.weight_map[name]
        except KeyError:
            raise KeyError(f"tensor {name} not in {self.dir}") from None
        f = self._files.get(fname)
        if f is None:
            f = self._files[fname] = SafeTensors(self.dir / fname)
        return f.get(name)

    def __contains__(self, name: str) -> bool:
        return name in self.weight_map


def save_file(tensors: dict[str, torch.Tensor], path: str | Path, metadata: dict | None = None) -> None:
    items = []
    for name, t in tensors.items():
        t = t.detach().to("cpu").contiguous()
        raw = t.view(torch.uint8) if t.dtype != torch.bool else t.to(torch.uint8)
        items.append((name, TORCH_TO_ST[t.dtype], list(t.shape), raw.numpy().reshape(-1)))
    runtime().write_safetensors(str(path), items, dict(metadata or {}))
