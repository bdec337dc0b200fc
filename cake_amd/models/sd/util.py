"""SD tensor packing (cake-core/src/models/sd/util.rs:8-63).

Several tensors travel as ONE 1-D f32 tensor:
``[n, ndim_0, dims_0..., data_0..., ndim_1, ...]`` — UNet sends
``[latents, text_embeddings, timestep]``, VAE ``[direction, x]`` with direction
1.0 = encode, 0.0 = decode.  Byte-compatible with the reference layout.
"""
from __future__ import annotations

import torch


def pack_tensors(tensors: list[torch.Tensor], device=None) -> torch.Tensor:
    device = device or tensors[0].device
    parts = [torch.tensor([float(len(tensors))], device=device)]
    for t in tensors:
        parts.append(torch.tensor([float(t.dim())], device=device))
        parts.append(torch.tensor([float(d) for d in t.shape], device=device))
        parts.append(t.reshape(-1).to(device=device, dtype=torch.float32))
    return torch.cat(parts)


def unpack_tensors(packed: torch.Tensor) -> list[torch.Tensor]:
    flat = packed.reshape(-1)
    head = flat[:1].tolist()
    n = int(head[0])
    out, idx = [], 1
    for _ in range(n):
        nd = int(flat[idx].item())
        idx += 1
        shape = [int(x) for x in flat[idx:idx + nd].tolist()]
        idx += nd
        numel = 1
        for d in shape:
            numel *= d
        out.append(flat[idx:idx + numel].reshape(shape))
        idx += numel
    return out
