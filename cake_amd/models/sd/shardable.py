"""SD shardable units (cake-core/src/models/sd/{sd_shardable,unet,vae,clip}.rs).

Every component — ``clip``, ``clip2``, ``vae``, ``unet`` — is a unit with the
reference's packed single-tensor interface so it can run locally or on a
worker (SingleOp with ``layer_name`` = component name):
* clip/clip2: token ids [1, 77] -> last hidden state [1, 77, D];
* unet: pack([latents, text_embeddings, t]) -> noise prediction;
* vae: pack([direction, x]) -> encode(x).sample() if direction == 1.0 else decode(x).
"""
from __future__ import annotations

import json
import logging
import os
from pathlib import Path

import torch

from .clip import ClipTextTransformer
from .config import SDConfig, get_config, mini_config, tiny_config
from .unet import UNet2DConditionModel
from .util import pack_tensors, unpack_tensors
from .vae import AutoencoderKL
from .weights import load_component, random_component, resolve

log = logging.getLogger("cake.sd")
SD_COMPONENTS = ("clip", "clip2", "vae", "unet")


def sd_config_for(ctx) -> SDConfig:
    a = ctx.args
    meta = Path(ctx.model_path) / "cake_sd.json"
    info = json.loads(meta.read_text()) if meta.exists() else {}
    if info.get("tiny", False) or info.get("mini", False):
        cfg = (mini_config if info.get("mini", False) else tiny_config)(a.sd_version)
        if a.sd_height:
            cfg.height = a.sd_height
        if a.sd_width:
            cfg.width = a.sd_width
        cfg.unet.sliced_attention_size = a.sd_sliced_attention_size
        return cfg
    return get_config(a.sd_version, a.sd_height, a.sd_width, a.sd_sliced_attention_size)


class SDUnit:
    def __init__(self, name: str, cfg: SDConfig, weights: dict[str, torch.Tensor], device, dtype):
        self.name, self.cfg, self.w, self.device, self.dtype = name, cfg, weights, device, dtype
        if name == "unet":
            self.model = UNet2DConditionModel(cfg.unet)
        elif name == "vae":
            self.model = AutoencoderKL(cfg.vae)
        else:
            self.model = ClipTextTransformer(cfg.clip if name == "clip" else cfg.clip2, weights)
        self.generator = torch.Generator(device="cpu")
        self._ctx = None  # (text embedding, cross-attention k/v cache) of the current generation
        self._graphs: dict = {}  # UNet step hipGraphs per input shape
        self.use_graph = (name == "unet" and torch.device(device).type == "cuda"
                          and os.environ.get("CAKE_SD_GRAPH", "1") != "0")

    def _kv_cache(self, emb: torch.Tensor) -> dict:
        """Cross-attention k/v of a text embedding are reused while it does not change
        (every step of one generation sends the same embedding)."""
        if self._ctx is not None:
            ref, cache = self._ctx
            if ref.shape == emb.shape and ref.dtype == emb.dtype and torch.equal(ref, emb):
                return cache
        cache: dict = {}
        self._ctx = (emb.clone(), cache)
        return cache

    def _unet_graph(self, lat: torch.Tensor, emb: torch.Tensor, t: float) -> torch.Tensor:
        """One UNet step as a hipGraph replay (captured on first use of a shape after one
        eager warm-up step that autotunes the convolutions).  The cross-attention
        k/v cache is refreshed in place when the text embedding changes."""
        from .unet import refresh_kv_cache
        key = (tuple(lat.shape), tuple(emb.shape), lat.dtype)
        st = self._graphs.get(key)
        if st is None:
            st = {"lat": lat.clone(), "emb": emb.clone(), "kv": {},
                  "t": torch.full((), t, device=lat.device, dtype=torch.float32)}
            self.model.forward(self.w, st["lat"], st["t"], st["emb"], kv_cache=st["kv"])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                st["out"] = self.model.forward(self.w, st["lat"], st["t"], st["emb"],
                                               kv_cache=st["kv"])
            st["graph"] = g
            self._graphs[key] = st
        elif not torch.equal(st["emb"], emb):
            st["emb"].copy_(emb)
            refresh_kv_cache(st["kv"], st["emb"])
        st["lat"].copy_(lat)
        st["t"].fill_(t)
        st["graph"].replay()
        return st["out"].clone()

    @torch.no_grad()
    def denoise(self, x: torch.Tensor, emb: torch.Tensor, sched, ts: list[int],
                guidance: float, use_guide: bool, seed: int, on_step=None) -> tuple:
        """Every diffusion step of ``ts`` on this local UNet, each step ONE hipGraph
        replay: time biases from the device timestep table -> UNet -> CFG combine +
        scheduler update + next UNet input (sd_small.hip) -> step += 1.  The first
        step runs eagerly (conv autotuning, cross-attention k/v) and the graph is
        captured from the second on; graphs are kept per shape / step count, their
        buffers refilled for a new generation.  on_step(i, x) runs between steps
        (intermediary images).  Returns (latents f32, per-step seconds)."""
        from ...ops import hip as K
        from .unet import refresh_kv_cache
        dev = self.device
        n = len(ts)
        x = x.to(dev, torch.float32).contiguous()
        emb = emb.to(dev, self.dtype).contiguous()
        B2 = x.shape[0] * (2 if use_guide else 1)
        key = ("denoise", tuple(x.shape), tuple(emb.shape), bool(use_guide), n, float(guidance))
        st = self._graphs.get(key)
        coef = torch.tensor([sched.step_coefs(t, ts[i + 1] if i + 1 < n else None)
                             for i, t in enumerate(ts)], dtype=torch.float32)
        ttab = torch.tensor([float(t) for t in ts], dtype=torch.float32)
        if st is None:
            st = {"x": x.clone(), "emb": emb.clone(), "kv": {}, "graph": None,
                  "t": ttab.to(dev), "coef": coef.to(dev),
                  "step": torch.zeros(1, dtype=torch.int32, device=dev),
                  "seed": torch.zeros(1, dtype=torch.int64, device=dev),
                  "inp": torch.empty((B2,) + tuple(x.shape[1:]), device=dev, dtype=self.dtype)}
            self._graphs[key] = st
        else:
            st["x"].copy_(x)
            st["t"].copy_(ttab)
            st["coef"].copy_(coef)
            st["step"].zero_()
            if not torch.equal(st["emb"], emb):
                st["emb"].copy_(emb)
                refresh_kv_cache(st["kv"], st["emb"])
        st["seed"].fill_(int(seed) & 0x7FFFFFFFFFFFFFFF)
        K.scale_copy(st["x"], sched.input_scale(ts[0]), use_guide, st["inp"])

        def body():
            pred = self.model.forward(self.w, st["inp"], st["t"], st["emb"], kv_cache=st["kv"],
                                      t_index=st["step"])
            K.sched_step(st["x"], pred, use_guide, guidance, st["coef"], st["step"],
                         st["seed"], next_in=st["inp"])
            K.step_advance(st["step"])
        evs = []
        for i in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if st["graph"] is not None and self.use_graph:
                st["graph"].replay()
            elif i == 0 or not self.use_graph:
                body()
            else:
                g = torch.cuda.CUDAGraph()
                # capture only records; the step is then replayed for real (guidance is
                # part of the key's graph: a new guidance value recaptures)
                with torch.cuda.graph(g):
                    body()
                st["graph"] = g
                g.replay()
            e1.record()
            evs.append((e0, e1))
            if on_step is not None:  # intermediary images: the host needs this step's x
                e1.synchronize()
                on_step(i, st["x"])
        # no host sync between steps otherwise: the next replay is enqueued while the
        # current one runs (a large graph's launch is not free)
        torch.cuda.synchronize()
        times = [a.elapsed_time(b) / 1e3 for a, b in evs]
        return st["x"].clone(), times

    def layer_name(self) -> str:
        return self.name

    def ident(self) -> str:
        return "local"

    @torch.no_grad()
    def forward_packed(self, x: torch.Tensor) -> torch.Tensor:
        if self.name in ("clip", "clip2"):
            return self.model.forward(x.to(self.device))
        parts = unpack_tensors(x.to(self.device))
        if self.name == "unet":
            lat, emb, t = parts
            emb = emb.to(self.dtype)
            if self.use_graph:
                return self._unet_graph(lat.to(self.dtype), emb, float(t.reshape(-1)[0]))
            return self.model.forward(self.w, lat.to(self.dtype), float(t.reshape(-1)[0]), emb,
                                      kv_cache=self._kv_cache(emb))
        direction, inp = parts
        inp = inp.to(self.dtype)
        if float(direction.reshape(-1)[0]) == 1.0:
            return self.model.encode(self.w, inp, self.generator)
        return self.model.decode(self.w, inp)

    # pipeline-facing helpers (same packing as the reference, unet.rs:81-100, vae.rs:87-108)
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward_packed(x)


class RemoteSDUnit:
    """A component served by a worker: SingleOp(layer_name=component, x=packed)."""

    def __init__(self, client, name: str):
        self.client, self.name = client, name

    def layer_name(self) -> str:
        return self.name

    def ident(self) -> str:
        return self.client.ident()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.client.forward_named(self.name, x)


def unet_forward_unpacked(unit, latents, text_embeddings, timestep: int, device) -> torch.Tensor:
    t = torch.tensor([float(timestep)], device=device)
    return unit.forward(pack_tensors([latents, text_embeddings, t], device))


def vae_encode(unit, image, device) -> torch.Tensor:
    return unit.forward(pack_tensors([torch.tensor([1.0], device=device), image], device))


def vae_decode(unit, latents, device) -> torch.Tensor:
    return unit.forward(pack_tensors([torch.tensor([0.0], device=device), latents], device))


def load_unit(name: str, ctx, cfg: SDConfig | None = None) -> SDUnit:
    a = ctx.args
    cfg = cfg or sd_config_for(ctx)
    override = {"unet": a.sd_unet, "vae": a.sd_vae, "clip": a.sd_clip, "clip2": a.sd_clip2}[name]
    if name == "clip2" and cfg.clip2 is None:
        raise ValueError(f"sd version {cfg.version} has no clip2")
    try:
        path = resolve(name, override, cfg.version, a.sd_use_f16, ctx.model_path)
        w = load_component(name, path, cfg, ctx.device, ctx.dtype)
        log.info("loaded %s from %s", name, path)
    except FileNotFoundError:
        if not getattr(a, "sd_random_init", False):
            raise
        log.warning("%s: no weights found, using random init", name)
        w = random_component(name, cfg, ctx.device, ctx.dtype)
    return SDUnit(name, cfg, w, ctx.device, ctx.dtype)


def load_sd_units(ctx, layers: list[str]) -> dict[str, SDUnit]:
    """Worker side (sd_shardable.rs:29-45): build each named component."""
    cfg = sd_config_for(ctx)
    units = {}
    for name in layers:
        if name not in SD_COMPONENTS:
            raise ValueError(f"unknown SD component {name!r} (clip, clip2, vae, unet)")
        units[name] = load_unit(name, ctx, cfg)
    return units
