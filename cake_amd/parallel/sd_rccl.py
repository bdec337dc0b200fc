"""Stable Diffusion over the device transport (``--transport rccl --model-type
image-model``, torchrun, one rank per GPU).

The reference places whole SD components on workers — ``clip``, ``clip2``,
``vae``, ``unet`` — and reaches each with one TCP round trip per call, packing
the tensors into one f32 buffer copied device -> host -> socket -> host ->
device (cake-core/src/models/sd/sd.rs:200-300, sd_shardable.rs:29-45,
unet.rs:81-100, util.rs:8-63).  Here rank 0 is the master (tokenizers,
scheduler, CFG, images, API) and rank i >= 1 serves topology node i's
components; a call is a small control message on a host channel (gloo) plus
the tensors moved device-to-device on the process group (RCCL over xGMI) — no
packing, no host copy of the data.

Beyond the reference:
* the UNet can be split over ranks by block group: ``unet.down.<i>``,
  ``unet.mid``, ``unet.up.<i>`` (``unet.down`` / ``unet.up`` = all of them);
  consecutive stages on one rank run as one hop (the text-model's
  contiguous-block batching), the skip stack travels with the feature map from
  rank to rank, and the text embedding reaches each stage owner once per
  generation (its cross-attention k/v are cached there);
* a UNet placed whole on one worker runs the entire denoising loop there (one
  hipGraph replay per step: UNet + CFG + scheduler, ``SDUnit.denoise``): one
  call per image instead of one round trip per step.
"""
from __future__ import annotations

import datetime
import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger("cake.sd.rccl")

_DT = {"float32": torch.float32, "float64": torch.float64, "float16": torch.float16,
       "bfloat16": torch.bfloat16,
       "int32": torch.int32, "int64": torch.int64, "uint8": torch.uint8}


class TensorLink:
    """Point-to-point tensor lists between two ranks: the metadata (shapes, dtypes) as
    an object on the host control group, the payloads on the data group (RCCL,
    device to device; host-staged when the data group is gloo)."""

    def __init__(self, device, ctrl, data=None):
        self.device, self.ctrl, self.data = torch.device(device), ctrl, data
        self.staged = dist.get_backend(data) == "gloo" and self.device.type == "cuda"

    def send(self, tensors: list, dst: int) -> None:
        meta = [(tuple(t.shape), str(t.dtype).replace("torch.", "")) for t in tensors]
        dist.send_object_list([meta], dst=dst, group=self.ctrl)
        for t in tensors:
            t = t.contiguous()
            dist.send(t.cpu() if self.staged else t, dst, group=self.data)

    def recv(self, src: int) -> list:
        box = [None]
        dist.recv_object_list(box, src=src, group=self.ctrl)
        out = []
        for shape, dt in box[0]:
            dev = "cpu" if self.staged else self.device
            t = torch.empty(shape, dtype=_DT[dt], device=dev)
            dist.recv(t, src, group=self.data)
            out.append(t.to(self.device) if self.staged else t)
        return out


def unet_stage_owners(topology, stages: list[str], world: int) -> dict[str, int]:
    """UNet stage -> rank (0 = master) from the topology (node i -> rank i + 1)."""
    own = {s: 0 for s in stages}
    for i, node in enumerate(topology.nodes):
        for name in node.layers:
            if name == "unet":
                sel = stages
            elif name in ("unet.down", "unet.up"):
                sel = [s for s in stages if s.startswith(name[5:] + ".")]
            elif name.startswith("unet."):
                if name[5:] not in stages:
                    raise ValueError(f"unknown UNet stage {name!r} (stages: {stages})")
                sel = [name[5:]]
            else:
                continue
            if i + 1 >= world:
                raise ValueError(f"topology node {node.name} has no rank (world {world})")
            for s in sel:
                own[s] = i + 1
    return own


def component_owner(topology, name: str, world: int) -> int:
    for i, node in enumerate(topology.nodes):
        if name in node.layers:
            if i + 1 >= world:
                raise ValueError(f"topology node {node.name} has no rank (world {world})")
            return i + 1
    return 0


def stage_runs(stages: list[str], owners: dict[str, int]) -> list[tuple[int, list[str]]]:
    runs: list[tuple[int, list[str]]] = []
    for s in stages:
        if runs and runs[-1][0] == owners[s]:
            runs[-1][1].append(s)
        else:
            runs.append((owners[s], [s]))
    return runs


class SDEngine:
    """Shared state of one rank: control group, link, placement."""

    def __init__(self, ctx, rank: int, world: int):
        from ..models.sd.shardable import sd_config_for
        from ..models.sd.unet import UNet2DConditionModel
        self.ctx, self.rank, self.world = ctx, rank, world
        self.device = ctx.device
        # the long timeout only on the control broadcast a worker idles in (serve());
        # a call's tensor metadata goes over a group with a normal timeout, so a master
        # waiting on a stuck worker fails instead of blocking for days
        idle = float(os.environ.get("CAKE_SERVE_IDLE_TIMEOUT", str(7 * 86400)))
        link_to = float(os.environ.get("CAKE_LINK_TIMEOUT", "600"))
        self.ctrl = dist.new_group(list(range(world)), backend="gloo",
                                   timeout=datetime.timedelta(seconds=idle))
        self.meta = dist.new_group(list(range(world)), backend="gloo",
                                   timeout=datetime.timedelta(seconds=link_to))
        self.link = TensorLink(self.device, self.meta)
        self.cfg = sd_config_for(ctx)
        self.stages = UNet2DConditionModel(self.cfg.unet).stage_names()
        topo = ctx.topology
        self.unet_owner = unet_stage_owners(topo, self.stages, world)
        self.runs = stage_runs(self.stages, self.unet_owner)
        names = ["clip", "vae"] + (["clip2"] if self.cfg.clip2 is not None else [])
        self.comp_owner = {n: component_owner(topo, n, world) for n in names}
        self.units: dict = {}
        self._emb, self._kv = None, {}   # worker: this generation's text embedding + k/v

    def unit(self, name: str):
        from ..models.sd.shardable import load_unit
        if name not in self.units:
            self.units[name] = load_unit(name, self.ctx, self.cfg)
        return self.units[name]

    def load_mine(self) -> None:
        """Load the components / UNet stages this rank serves (workers)."""
        for n, r in self.comp_owner.items():
            if r == self.rank:
                self.unit(n)
        if any(r == self.rank for r in self.unet_owner.values()):
            self.unit("unet")

    def ctrl_send(self, cmd: dict) -> None:
        dist.broadcast_object_list([cmd], src=0, group=self.ctrl)

    def ctrl_recv(self) -> dict:
        box = [None]
        dist.broadcast_object_list(box, src=0, group=self.ctrl)
        return box[0]

    # ------------------------------------------------------------------ worker
    def serve(self) -> None:
        """Worker loop: run what the master announces until ``stop``."""
        while True:
            cmd = self.ctrl_recv()
            op = cmd["op"]
            if op == "stop":
                return
            if op == "call" and cmd["rank"] == self.rank:
                args = self.link.recv(0)
                self.link.send(self._call(cmd["unit"], cmd["method"], args, cmd), 0)
            elif op == "unet":
                self._serve_unet_step(cmd)
            elif op == "denoise" and cmd["rank"] == self.rank:
                x, emb = self.link.recv(0)
                lat, times = self._denoise(x, emb, cmd)
                self.link.send([lat, torch.tensor(times, dtype=torch.float64,
                                                  device=self.device)], 0)

    @torch.no_grad()
    def _call(self, name: str, method: str, args: list, cmd: dict) -> list:
        u = self.unit(name)
        if method == "clip":
            return [u.model.forward(args[0])]
        if method == "vae_encode":
            return [u.model.encode(u.w, args[0].to(u.dtype), u.generator)]
        if method == "vae_decode":
            return [u.model.decode(u.w, args[0].to(u.dtype))]
        raise ValueError(f"unknown method {method}")

    @torch.no_grad()
    def _serve_unet_step(self, cmd: dict) -> None:
        mine = [(j, names) for j, (r, names) in enumerate(self.runs) if r == self.rank]
        if not mine:
            return
        u = self.unit("unet")
        if cmd["emb_new"]:
            self._emb = self.link.recv(0)[0]
            self._kv = {}
        for j, names in mine:
            prev = self.runs[j - 1][0] if j > 0 else 0
            nxt = self.runs[j + 1][0] if j + 1 < len(self.runs) else 0
            state = self.link.recv(prev)
            x, skips = u.model.forward_stages(u.w, names, state[0], state[1:], cmd["t"],
                                              self._emb, kv_cache=self._kv)
            self.link.send([x] + skips, nxt)

    def _denoise(self, x, emb, cmd):
        from ..models.sd.schedulers import build_scheduler
        u = self.unit("unet")
        sched = build_scheduler(self.cfg.scheduler, cmd["n_steps"])
        return u.denoise(x, emb, sched, cmd["ts"], cmd["guidance"], cmd["use_guide"],
                         cmd["seed"])

    # ------------------------------------------------------------------ master
    def shutdown(self) -> None:
        self.ctrl_send({"op": "stop"})


class RemoteComponent:
    """Master-side proxy of a clip / clip2 / vae served by another rank (same call
    interface as the local SDUnit: ``forward(packed)`` for vae, ids for clip)."""

    def __init__(self, eng: SDEngine, name: str, rank: int):
        self.eng, self.name, self.rank = eng, name, rank

    def layer_name(self) -> str:
        return self.name

    def ident(self) -> str:
        return f"rank{self.rank}"

    def _rpc(self, method: str, args: list) -> torch.Tensor:
        e = self.eng
        e.ctrl_send({"op": "call", "rank": self.rank, "unit": self.name, "method": method})
        e.link.send(args, self.rank)
        return e.link.recv(self.rank)[0]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.name in ("clip", "clip2"):
            return self._rpc("clip", [x.to(self.eng.device)])
        from ..models.sd.util import unpack_tensors
        direction, inp = unpack_tensors(x.to(self.eng.device))
        m = "vae_encode" if float(direction.reshape(-1)[0]) == 1.0 else "vae_decode"
        return self._rpc(m, [inp.to(self.eng.ctx.dtype)])


class DeviceUNet:
    """Master-side UNet over the ranks that own its stages.  ``forward(packed)`` is
    one step (the reference's per-step round trip, generalised to a chain of stage
    owners); ``denoise`` runs the whole loop on the owner when one worker holds the
    entire UNet."""

    def __init__(self, eng: SDEngine):
        self.eng = eng
        self.name = "unet"
        owners = set(eng.unet_owner.values())
        self.whole_rank = owners.pop() if len(owners) == 1 else None
        self._emb = None

    @property
    def can_denoise(self) -> bool:
        return self.whole_rank not in (None, 0) and self.eng.device.type == "cuda"

    def layer_name(self) -> str:
        return "unet"

    def ident(self) -> str:
        return "rccl"

    @torch.no_grad()
    def forward(self, packed: torch.Tensor) -> torch.Tensor:
        from ..models.sd.util import unpack_tensors
        e = self.eng
        lat, emb, t = unpack_tensors(packed.to(e.device))
        dt = e.ctx.dtype
        lat, emb = lat.to(dt), emb.to(dt)
        new = self._emb is None or self._emb.shape != emb.shape or not torch.equal(self._emb, emb)
        if new:
            self._emb = emb.clone()
            self._kv = {}
        tt = float(t.reshape(-1)[0])
        e.ctrl_send({"op": "unet", "t": tt, "emb_new": new})
        if new:
            for r in sorted({r for r, _ in e.runs if r != 0}):
                e.link.send([emb], r)
        x, skips = lat, []
        holder = 0
        for j, (r, names) in enumerate(e.runs):
            if r == 0:
                if holder != 0:
                    st = e.link.recv(holder)
                    x, skips = st[0], st[1:]
                u = e.unit("unet")
                x, skips = u.model.forward_stages(u.w, names, x, skips, tt, self._emb,
                                                  kv_cache=self._kv)
                holder = 0
            else:
                if holder == 0:
                    e.link.send([x] + skips, r)
                holder = r
        if holder != 0:
            x = e.link.recv(holder)[0]
        return x

    @torch.no_grad()
    def denoise(self, x, emb, sched, ts, guidance, use_guide, seed, on_step=None):
        e = self.eng
        e.ctrl_send({"op": "denoise", "rank": self.whole_rank, "ts": [int(t) for t in ts],
                     "n_steps": sched.n_steps,
                     "guidance": float(guidance), "use_guide": bool(use_guide),
                     "seed": int(seed)})
        e.link.send([x.to(e.device, torch.float32), emb.to(e.device, e.ctx.dtype)],
                    self.whole_rank)
        lat, times = e.link.recv(self.whole_rank)
        return lat, times.cpu().tolist()


def native_split_owners(topology, cfg, world: int) -> list[int] | None:
    """Stage -> rank of the native engine's split UNet (csrc/engine/sd_engine.cpp
    CakeSdSplitOpts) for a topology that places only UNet stages on ranks >= 1, in
    contiguous runs 0, 1, 2, ... in stage order; None when the topology needs the Python
    transport (a text encoder or the VAE on a worker rank, or another stage order) or
    places nothing."""
    n = len(cfg.unet.blocks)
    stages = [f"down.{i}" for i in range(n)] + ["mid"] + [f"up.{i}" for i in range(n)]
    for comp in ("clip", "clip2", "vae"):
        if component_owner(topology, comp, world) != 0:
            return None
    own = unet_stage_owners(topology, stages, world)
    owners = [own[s] for s in stages]
    if max(owners) == 0 or owners[0] != 0:
        return None
    for a, b in zip(owners, owners[1:]):
        if b not in (a, a + 1):
            return None
    return owners


def run_native_split(ctx, owners: list[int]) -> None:
    """Every rank opens the native SD engine's split UNet (one process per GPU, device bulk
    hops, TCP control plane on MASTER_PORT + 2); rank 0 is the master (CLI images or the
    REST API over NativeSDGenerator), the others serve its denoise steps."""
    from ..models.sd.native_generator import NativeSDGenerator
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    addr = (f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}:"
            f"{int(os.environ.get('MASTER_PORT', '29500')) + 2}")
    timeout = float(os.environ.get("CAKE_HOP_TIMEOUT", "60"))
    split = dict(rank=rank, world=world, master_addr=addr, owners=owners,
                 hop_timeout_s=timeout)
    log.info("rank %d/%d: native split UNet, stage owners %s", rank, world, owners)
    # the same model resolution on every rank; ranks > 0 load the UNet only (the engine)
    gen = NativeSDGenerator.load(ctx, split=split)
    try:
        if rank == 0:
            from ..master import Master
            Master(ctx, sd=gen).run()
        else:
            gen.eng.serve()
    finally:
        gen.eng.close()


def run_sd_rccl(ctx) -> None:
    """Entry of ``--transport rccl --model-type image-model`` (every rank): the native
    engine's split UNet when the topology places UNet stages only, in runs over ranks in
    stage order (CAKE_NATIVE=0 or any other placement: the Python transport below)."""
    from .rccl_roles import _init_dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    from ..models.sd.native_generator import native_sd_eligible
    if world > 1 and native_sd_eligible(ctx):
        from ..models.sd.shardable import sd_config_for
        owners = native_split_owners(ctx.topology, sd_config_for(ctx), world)
        if owners is not None:
            run_native_split(ctx, owners)
            return
    _init_dist(ctx, rank, world)
    try:
        eng = SDEngine(ctx, rank, world)
        log.info("rank %d/%d: components %s, unet stages %s", rank, world,
                 [n for n, r in eng.comp_owner.items() if r == rank],
                 [s for s, r in eng.unet_owner.items() if r == rank])
        if rank != 0:
            eng.load_mine()
            dist.barrier()
            eng.serve()
        else:
            from ..master import Master
            from ..models.sd.pipeline import SDGenerator

            def remote(name):
                if name == "unet":
                    if all(r == 0 for r in eng.unet_owner.values()):
                        return None
                    return DeviceUNet(eng)
                r = eng.comp_owner.get(name, 0)
                return RemoteComponent(eng, name, r) if r != 0 else None
            sd = SDGenerator.load(ctx, remote=remote)
            dist.barrier()
            try:
                Master(ctx, sd=sd).run()
            finally:
                eng.shutdown()
        dist.barrier()
    finally:
        dist.destroy_process_group()
