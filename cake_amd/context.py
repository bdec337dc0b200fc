"""Process-wide context (cake-core/src/cake/mod.rs:38-101 ``Context::from_args``).

dtype: f16 by default, f16/bf16/f32 accepted (mod.rs:54-60); device: GPU
``--device`` unless ``--cpu`` (utils/mod.rs:15-30); topology loaded for the
model type (an empty file means everything local); generation/sampling
parameters from the CLI flags.
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass, field
from pathlib import Path

import torch

from .models.sampling import SamplingConfig
from .parallel.topology import Topology

log = logging.getLogger("cake")


def inference_device(cpu: bool, ordinal: int) -> torch.device:
    if not cpu and torch.cuda.is_available():
        torch.cuda.set_device(ordinal)
        return torch.device("cuda", ordinal)
    return torch.device("cpu")


@dataclass
class Context:
    args: object
    mode: str = "master"
    name: str | None = None
    address: str = "127.0.0.1:10128"
    model_path: Path = Path(".")
    model_type: str = "text-model"
    topology: Topology = field(default_factory=Topology.empty)
    device: torch.device = torch.device("cpu")
    dtype: torch.dtype = torch.float16
    sampling: SamplingConfig = field(default_factory=SamplingConfig)
    max_seq_len: int = 4096
    no_graph: bool = False

    @classmethod
    def from_args(cls, args) -> "Context":
        from .models.llama3.factory import parse_dtype
        dtype = parse_dtype(args.dtype or "f16")
        device = inference_device(args.cpu, args.device)
        if device.type == "cpu" and dtype != torch.float32:
            log.info("CPU mode: computing in f32")
            dtype = torch.float32
        text = args.model_type == "text-model"
        topo_path = Path(args.topology)
        if topo_path.exists():
            topology = Topology.from_path(str(topo_path), text_model=text)
        else:
            if args.mode == "worker":
                raise FileNotFoundError(f"topology {topo_path} not found")
            log.warning("topology %s not found: everything runs locally", topo_path)
            topology = Topology.empty()
        sampling = SamplingConfig(temperature=args.temperature, top_k=args.top_k, top_p=args.top_p,
                                  repeat_penalty=args.repeat_penalty,
                                  repeat_last_n=args.repeat_last_n, seed=args.seed)
        return cls(args=args, mode=args.mode, name=args.name, address=args.address,
                   model_path=Path(args.model), model_type=args.model_type, topology=topology,
                   device=device, dtype=dtype, sampling=sampling, max_seq_len=args.max_seq_len,
                   no_graph=getattr(args, "no_graph", False))


def hbm_mib(device=None) -> dict:
    """HBM of this rank's GPU: torch-allocated now / peak and device-wide used (MiB)."""
    import torch
    if not torch.cuda.is_available():
        return {}
    dev = torch.cuda.current_device() if device is None else device
    free, total = torch.cuda.mem_get_info(dev)
    return {"hbm_alloc_mib": round(torch.cuda.memory_allocated(dev) / 2**20, 1),
            "hbm_peak_mib": round(torch.cuda.max_memory_allocated(dev) / 2**20, 1),
            "hbm_used_mib": round((total - free) / 2**20, 1),
            "hbm_total_mib": round(total / 2**20, 1)}


def rss_mib() -> float:
    try:
        with open(f"/proc/{os.getpid()}/status") as f:
            for line in f:
                if line.startswith("VmRSS:"):
                    return int(line.split()[1]) / 1024
    except OSError:
        pass
    return float("nan")
