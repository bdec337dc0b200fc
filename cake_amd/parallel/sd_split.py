"""Split-UNet diffusion over N ranks: BASELINE config 5 ("SDXL UNet blocks sharded
across workers") as a measured path.

The reference reaches a remote UNet once per diffusion step — the latents, text
embedding and timestep packed into one f32 buffer and copied device -> host ->
socket -> host -> device each way (cake-core/src/models/sd/sd.rs:464-513, the
per-step time including that round trip at :506-507; unet.rs:81-100 packing;
sd_shardable.rs:29-45 dispatch).  Here the UNet's block groups (``down.i``,
``mid``, ``up.i``: UNet2DConditionModel.stage_names) are spread over the ranks
contiguously, and one diffusion step walks them in order (:class:`SplitPlan`): the
running feature map follows the runs and returns to rank 0, and every skip tensor of
the down path goes ONCE from the rank that pushed it straight to the rank whose up
stage pops it (the full-resolution down.0 skips never cross the ranks in between, and
their transfer overlaps those ranks' compute).

Transport: on the GPU every step after the first is ONE hipGraph replay per rank —
receive(s), its stages, send(s), and on rank 0 the CFG combine + scheduler update —
with the hops as device bulk copies into the receiver's HBM (IPC-mapped inbox, flag
word; parallel/hop.py BulkInbox / BulkPeer) and no per-step host work at all
(:class:`_DeviceChannels`).  The first step runs eagerly over :class:`PackedLink`
(RCCL / gloo, one packed buffer per message), which also fixes the message layouts.
The text embedding reaches each stage owner once; the cross-attention k/v of it are
cached there for every step.  Rank 0 (the master) owns the first stages.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

_DT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}


class PackedLink:
    """Fixed-signature tensor lists between ranks as one packed buffer per hop.

    The first send of a (peer, key) signature ships the shapes and dtype as a host
    object on `meta` (a gloo group); every later hop of that signature is one
    ``dist.send`` of the packed payload on `data` (RCCL: device to device, ordered on
    the current stream) with no host round trip.  All tensors of one list share a
    dtype (the UNet state is the model dtype).  Received tensors are views into a
    per-signature buffer that the next receive of the same signature overwrites.
    """

    def __init__(self, device, meta, data=None):
        self.device, self.meta, self.data = torch.device(device), meta, data
        self.staged = dist.get_backend(data) == "gloo" and self.device.type == "cuda"
        self._sent: dict = {}
        self._recv: dict = {}
        self._bufs: dict = {}

    @staticmethod
    def _sig(tensors: list) -> tuple:
        dts = {t.dtype for t in tensors}
        if len(dts) != 1:
            raise ValueError(f"PackedLink: one dtype per list, got {dts}")
        return (str(tensors[0].dtype).replace("torch.", ""),
                tuple(tuple(t.shape) for t in tensors))

    def _buf(self, key, numel: int, dtype) -> torch.Tensor:
        b = self._bufs.get(key)
        if b is None or b.numel() != numel or b.dtype != dtype:
            dev = "cpu" if self.staged else self.device
            b = self._bufs[key] = torch.empty(numel, dtype=dtype, device=dev)
        return b

    def send(self, tensors: list, dst: int, key: str) -> None:
        sig = self._sig(tensors)
        if self._sent.get((dst, key)) != sig:
            dist.send_object_list([sig], dst=dst, group=self.meta)
            self._sent[(dst, key)] = sig
        if len(tensors) == 1 and tensors[0].is_contiguous() and not self.staged:
            buf = tensors[0].reshape(-1)
        else:
            n = sum(t.numel() for t in tensors)
            buf = self._buf(("s", dst, key), n, tensors[0].dtype)
            o = 0
            for t in tensors:
                buf[o:o + t.numel()].view(t.shape).copy_(t)
                o += t.numel()
        dist.send(buf, dst, group=self.data)

    def recv(self, src: int, key: str) -> list:
        sig = self._recv.get((src, key))
        if sig is None:
            box = [None]
            dist.recv_object_list(box, src=src, group=self.meta)
            sig = self._recv[(src, key)] = box[0]
        dt, shapes = sig
        n = 0
        for s in shapes:
            n += int(torch.Size(s).numel())
        buf = self._buf(("r", src, key), n, _DT[dt])
        dist.recv(buf, src, group=self.data)
        if self.staged:
            buf = buf.to(self.device)
        out, o = [], 0
        for s in shapes:
            k = int(torch.Size(s).numel())
            out.append(buf[o:o + k].view(s))
            o += k
        return out

    def forget(self, peer: int, key: str) -> None:
        """Drop a signature (the next hop of it re-sends its shapes)."""
        self._sent.pop((peer, key), None)
        self._recv.pop((peer, key), None)


def stage_costs(ucfg, h: int, w: int) -> dict[str, float]:
    """Forward FLOPs of each UNet stage (down.i, mid, up.i) for an h x w latent, batch 1:
    3x3 convolutions, the resnets' 1x1 shortcuts, and per transformer block the
    projections (self q|k|v|o 4C^2, cross q|o 2C^2, GEGLU FF 12C^2, proj in/out 2C^2 per
    model) plus the attention products (self HW^2 C, cross 77 HW C).  Only the ratios
    matter: they balance the split."""
    blocks = list(ucfg.blocks)
    L = ucfg.layers_per_block

    def conv(cin, cout, hw, k=3):
        return 2.0 * k * k * cin * cout * hw

    def resnet(cin, cout, hw):
        return conv(cin, cout, hw) + conv(cout, cout, hw) + (conv(cin, cout, hw, 1) if cin != cout else 0)

    def transformer(c, hw, depth):
        per = 2.0 * hw * c * c * (4 + 2 + 12) + 4.0 * hw * hw * c + 4.0 * hw * 77 * c
        return depth * per + 2 * 2.0 * hw * c * c

    costs: dict[str, float] = {}
    hw = h * w
    chans = [b.out_channels for b in blocks]
    cin = chans[0]
    for i, b in enumerate(blocks):
        c = conv(ucfg.in_channels, chans[0], hw) if i == 0 else 0.0
        for j in range(L):
            c += resnet(cin if j == 0 else b.out_channels, b.out_channels, hw)
            if b.cross_attn:
                c += transformer(b.out_channels, hw, b.transformer_layers)
        cin = b.out_channels
        if i < len(blocks) - 1:
            hw //= 4
            c += conv(b.out_channels, b.out_channels, hw)
        costs[f"down.{i}"] = c
    cm, mb = chans[-1], blocks[-1]
    costs["mid"] = 2 * resnet(cm, cm, hw) + transformer(cm, hw, mb.transformer_layers)
    rev = list(reversed(chans))
    out = rev[0]
    for i, b in enumerate(reversed(blocks)):
        prev, out = out, rev[i]
        skip_in = rev[min(i + 1, len(rev) - 1)]
        c = 0.0
        for j in range(L + 1):
            skip = skip_in if j == L else out
            c += resnet((prev if j == 0 else out) + skip, out, hw)
            if b.cross_attn:
                c += transformer(out, hw, b.transformer_layers)
        if i < len(blocks) - 1:
            hw *= 4
            c += conv(out, out, hw)
        else:
            c += conv(out, ucfg.out_channels, hw)
        costs[f"up.{i}"] = c
    return costs


def split_stages(stages: list[str], world: int,
                 costs: dict[str, float] | None = None) -> list[tuple[int, list[str]]]:
    """Contiguous runs of UNet stages over min(world, len(stages)) ranks, rank 0 first
    (the master owns the UNet input side).  With `costs` the split minimises the largest
    rank's cost (the per-step critical path of the sequential pipeline); else it is
    balanced by stage count."""
    n = min(world, len(stages))
    if costs is None:
        runs, s = [], 0
        for r in range(n):
            e = s + (len(stages) - s) // (n - r)
            runs.append((r, stages[s:e]))
            s = e
        return runs
    c = [float(costs[x]) for x in stages]
    m = len(c)
    pre = [0.0]
    for x in c:
        pre.append(pre[-1] + x)
    INF = float("inf")
    # best[k][j]: min over splits of stages[:j] into k non-empty runs of the largest run
    best = [[INF] * (m + 1) for _ in range(n + 1)]
    cut = [[0] * (m + 1) for _ in range(n + 1)]
    best[0][0] = 0.0
    for k in range(1, n + 1):
        for j in range(k, m - (n - k) + 1):
            for i in range(k - 1, j):
                v = max(best[k - 1][i], pre[j] - pre[i])
                if v < best[k][j]:
                    best[k][j], cut[k][j] = v, i
    bounds, j = [], m
    for k in range(n, 0, -1):
        i = cut[k][j]
        bounds.append((i, j))
        j = i
    bounds.reverse()
    return [(r, stages[a:b]) for r, (a, b) in enumerate(bounds)]


def skip_counts(model) -> dict[str, tuple[int, int]]:
    """(pushed, popped) skip tensors of each UNet stage (UNet2DConditionModel.run_stage):
    down.0 pushes conv_in's output, every down stage one per resnet plus its downsampler's,
    every up stage pops one per resnet."""
    counts: dict[str, tuple[int, int]] = {}
    for i, (res, _, ds) in enumerate(model.down):
        counts[f"down.{i}"] = ((1 if i == 0 else 0) + len(res) + (1 if ds is not None else 0), 0)
    counts["mid"] = (0, 0)
    for i, (res, _, _) in enumerate(model.up):
        counts[f"up.{i}"] = (0, len(res))
    return counts


class SplitPlan:
    """Who sends what to whom in one split-UNet step.

    The feature map x follows the runs (rank of run j -> rank of run j+1, the last back
    to rank 0 as the UNet output).  Each skip tensor goes ONCE, from the rank whose down
    stage pushed it straight to the rank whose up stage pops it — not relayed through the
    ranks in between (the reference has one remote UNet, sd.rs:464-513; here the largest
    skips, down.0's full-resolution maps, would otherwise cross every hop).  A channel
    (a, b) carries one message per step: items "x" and / or skip indices (push order)."""

    def __init__(self, stages: list[str], counts: dict[str, tuple[int, int]], runs: list):
        self.runs = runs
        self.order = [r for r, _ in runs]
        owner = {n: r for r, names in runs for n in names}
        producer, consumer, stack, k = {}, {}, [], 0
        self.base: dict[int, int] = {}
        for n in stages:
            push, pop = counts[n]
            if push:
                self.base.setdefault(owner[n], k)
            for _ in range(pop):
                consumer[stack.pop()] = owner[n]
            for _ in range(push):
                producer[k] = owner[n]
                stack.append(k)
                k += 1
        if stack:
            raise ValueError(f"unbalanced skip stack: {stack}")
        self.producer, self.consumer = producer, consumer
        self.channels: dict[tuple[int, int], list] = {}
        for j, r in enumerate(self.order[:-1]):
            self.channels[(r, self.order[j + 1])] = ["x"]
        if len(self.order) > 1:
            self.channels[(self.order[-1], self.order[0])] = ["x"]  # the UNet output
        for i in sorted(producer):
            a, b = producer[i], consumer[i]
            if a != b:
                self.channels.setdefault((a, b), []).append(i)

    def incoming(self, rank: int) -> list[tuple[int, list]]:
        """(source, items) of this rank's messages in receive order: the feature map's
        source first, then the skip-only sources."""
        ins = [(a, it) for (a, b), it in self.channels.items() if b == rank]
        return sorted(ins, key=lambda e: ("x" not in e[1], e[0]))

    def outgoing(self, rank: int) -> list[tuple[int, list]]:
        """(destination, items) in send order: the feature map's destination first (the
        critical path), then the skip-only destinations."""
        outs = [(b, it) for (a, b), it in self.channels.items() if a == rank]
        return sorted(outs, key=lambda e: ("x" not in e[1], e[0]))

    def received_skips(self, rank: int) -> list[int]:
        return sorted(i for i, c in self.consumer.items()
                      if c == rank and self.producer[i] != rank)

    def step(self, rank: int, x, run_stages, recv, send):
        """One step on `rank`: receive, run the stages, send.  run_stages(x, skips) ->
        (x, skips) is the stage run; recv(src) -> {item: tensor}; send(dst, items,
        tensors).  Returns the UNet output on rank 0 (x of the last run), else None."""
        got: dict = {}
        for a, _ in self.incoming(rank) if rank != self.order[0] else []:
            got.update(recv(a))
        if rank != self.order[0]:
            x = got.pop("x")
        skips = [got[i] for i in self.received_skips(rank)]
        x, rest = run_stages(x, skips)
        base = self.base.get(rank, 0)
        own = {base + i: t for i, t in enumerate(rest)}
        for b, items in self.outgoing(rank):
            send(b, items, [x if it == "x" else own[it] for it in items])
        if rank == self.order[0]:
            if len(self.order) == 1:
                return x
            out = recv(self.order[-1])
            return out["x"]
        return None


def _sched_update(x, pred, coef_row, guidance: float):
    """Host-math CFG combine + scheduler update (the CPU / gloo plumbing path; the
    device path is sd_small.hip sched_step): x <- A x + B eps (noise term omitted)."""
    A, B = float(coef_row[0]), float(coef_row[1])
    u, c = pred.float().chunk(2)
    eps = u + guidance * (c - u)
    return A * x + B * eps


@torch.no_grad()
def measure_sd_split(env, steps: int = 4, warmup: int = 2, version: str = "xl",
                     dtype=torch.float16, tiny: bool = False) -> dict | None:
    """Seconds per diffusion step of one image (CFG batch 2) with the UNet split by
    block group over the ranks of `env` (pipeline_bench.DistEnv).  Every rank builds
    the same random-init UNet (seeded) and keeps the weights of its stages; rank 0
    returns the record (None elsewhere)."""
    from ..models.sd.config import get_config, tiny_config
    from ..models.sd.schedulers import build_scheduler
    from ..models.sd.unet import UNet2DConditionModel
    from ..models.sd.weights import random_component_on_device, unet_stage_keep

    rank, world, dev = env.rank, env.world, env.dev
    cfg = tiny_config(version) if tiny else get_config(version)
    model = UNet2DConditionModel(cfg.unet)
    stages = model.stage_names()
    runs = split_stages(stages, world, stage_costs(cfg.unet, cfg.height // 8, cfg.width // 8))
    mine = [names for r, names in runs if r == rank]
    names = mine[0] if mine else []
    hip = dev.type == "cuda"
    if not hip:
        dtype = torch.float32
    meta = dist.new_group(list(range(world)), backend="gloo")
    t_load = time.perf_counter()
    err = None
    try:
        W = random_component_on_device("unet", cfg, dev, dtype, seed=7,
                                       keep=unet_stage_keep(names, len(stages)))
        if hip:
            torch.cuda.synchronize(dev)
    except Exception as e:  # noqa: BLE001  (reported to every rank below)
        err = f"rank {rank}: {type(e).__name__}: {e}"[:300]
    # a setup failure on ONE rank (e.g. an OOM drawing its stage weights) must stop every
    # rank before the step loop, not leave the peers blocked in a hop receive
    oks: list = [None] * world
    dist.all_gather_object(oks, err, group=meta)
    bad = [x for x in oks if x]
    if bad:
        raise RuntimeError("split-UNet setup failed: " + "; ".join(bad))
    load_s = time.perf_counter() - t_load
    link = PackedLink(dev, meta, None)
    plan = SplitPlan(stages, skip_counts(model), runs)
    g = torch.Generator(device="cpu").manual_seed(11)
    emb = torch.randn(2, 77, cfg.unet.cross_attention_dim, generator=g).to(dev, dtype)
    lat = torch.randn(1, 4, cfg.height // 8, cfg.width // 8, generator=g).to(dev)
    n_steps = warmup + steps
    sched = build_scheduler(cfg.scheduler, n_steps + 1)
    ts = sched.timesteps()[:n_steps]
    coef = torch.tensor([sched.step_coefs(t, ts[i + 1] if i + 1 < n_steps else None)
                         for i, t in enumerate(ts)], dtype=torch.float32)
    kv: dict = {}
    last = len(runs) - 1
    my_run = next((j for j, (r, _) in enumerate(runs) if r == rank), None)
    inp = torch.empty(2, *lat.shape[1:], device=dev, dtype=dtype)
    x = lat.clone() * sched.init_noise_sigma
    step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
    seed_dev = torch.zeros(1, dtype=torch.int64, device=dev)
    coef_dev = coef.to(dev)
    # (one spare entry: compute-only replays after the last step read index n_steps)
    ttab = torch.tensor([float(t) for t in ts] + [float(ts[-1])], dtype=torch.float32,
                        device=dev)
    device_hops = (hip and world > 1 and len(runs) > 1 and warmup >= 1
                   and os.environ.get("CAKE_SD_SPLIT_DEVICE", "1") != "0")
    compute_s: list[float] = []
    step_s: list[float] = []
    tcur = [0.0, 0]
    timing = [False]  # eager steps: time the stage compute inline

    def sync():
        if hip:
            torch.cuda.synchronize(dev)

    def run_stages(x_, skips_):
        if timing[0]:
            sync()
            c0 = time.perf_counter()
        if hip:  # device timestep table indexed on the device (graph-replayable)
            out = model.forward_stages(W, names, x_, skips_, ttab, emb, kv_cache=kv,
                                       t_index=step_dev)
        else:
            out = model.forward_stages(W, names, x_, skips_, tcur[0], emb, kv_cache=kv)
        if timing[0]:
            sync()
            compute_s.append(time.perf_counter() - c0)
        return out

    def key(a, b):
        return f"c{a}>{b}"

    def recv_packed(a):
        return dict(zip(plan.channels[(a, rank)], link.recv(a, key(a, rank))))

    def send_packed(b, items, tensors):
        link.send(tensors, b, key(rank, b))

    def after(pred):
        """rank 0: CFG combine + scheduler update (+ the next step's UNet input)."""
        nonlocal x
        if hip:
            from ..ops import hip as K
            K.sched_step(x, pred, True, 7.5, coef_dev, step_dev, seed_dev, next_in=inp)
        else:
            x = _sched_update(x, pred, coef[int(tcur[1])], 7.5)

    def eager_step(i):
        tcur[0], tcur[1] = float(ts[i]), i
        if rank == 0 and not hip:
            inp.copy_((x * sched.input_scale(ts[i])).expand(2, -1, -1, -1))
        if my_run is not None:
            pred = plan.step(rank, inp if rank == 0 else None, run_stages, recv_packed,
                             send_packed)
            if rank == 0:
                after(pred)
        if hip:
            from ..ops import hip as K
            K.step_advance(step_dev)

    if hip:
        from ..ops import hip as K
        K.scale_copy(x, sched.input_scale(ts[0]), True, inp)
    dist.barrier()
    chan = None
    for i in range(n_steps):
        if device_hops and i == 1:
            sync()
            chan = _DeviceChannels(plan, rank, link, meta, dev, key)
            break
        sync()
        t0 = time.perf_counter()
        timing[0] = i >= warmup
        eager_step(i)
        timing[0] = False
        sync()
        if i >= warmup:
            step_s.append(time.perf_counter() - t0)
    if chan is not None:
        try:
            step_s, compute_s = chan.run(plan, rank, world, my_run, run_stages, inp, after,
                                         step_dev, n_steps - 1, warmup - 1)
        finally:
            chan.close(meta)
    sync()
    comp = [0.0] * world
    allc = [None] * world
    dist.all_gather_object(allc, (rank, sum(compute_s) / max(1, len(compute_s)), load_s))
    for r_, c_, _ in allc:
        comp[r_] = c_
    dist.barrier()
    if rank != 0:
        return None
    per_step = sum(step_s) / max(1, len(step_s))
    hops = len(runs)  # runs - 1 forward hops of the feature map + the output back
    comp_sum = sum(comp)
    if chan is not None:
        transport = ("device bulk hops: IPC peer stores into the next rank's HBM inside each "
                     "rank's step hipGraph, skips routed producer -> consumer")
    elif hip:
        transport = ("gloo, host-staged packed buffer per hop" if link.staged else
                     "rccl p2p, packed buffer per hop") + ", skips routed producer -> consumer"
    else:
        transport = "gloo"
    return {"seconds_per_step": round(per_step, 5), "version": version,
            "resolution": f"{cfg.width}x{cfg.height}", "batch": 2,
            "dtype": {torch.float16: "f16", torch.bfloat16: "bf16",
                      torch.float32: "f32"}[dtype],
            "ranks_used": len(runs), "stages": {f"rank{r}": n for r, n in runs},
            "compute_s_per_rank": [round(c, 5) for c in comp],
            "hops_per_step": hops,
            "channels": {f"{a}->{b}": [str(it) for it in items]
                         for (a, b), items in plan.channels.items()},
            "hop_bytes": chan.bytes_per_channel() if chan is not None else None,
            "hop_us_mean": round(max(0.0, per_step - comp_sum) / hops * 1e6, 1) if hops else 0.0,
            "steps": steps, "warmup": warmup,
            "per_step_s": [round(s, 5) for s in step_s],
            # the final latents (equivalence across rank counts; tests)
            "latent_checksum": float(x.double().sum()), "latent_abs": float(x.double().abs().sum()),
            "transport": transport}


def _layout(tensors_or_sig) -> tuple[list[int], int]:
    """16-byte aligned offsets of a message's items and its size."""
    offs, o = [], 0
    for nbytes in tensors_or_sig:
        offs.append(o)
        o += (int(nbytes) + 15) // 16 * 16
    return offs, max(o, 16)


class _DeviceChannels:
    """The split-UNet step on device hops (parallel/hop.py BulkInbox / BulkPeer): each
    rank's step — receive(s), its stages, send(s), and on rank 0 the scheduler update —
    is ONE hipGraph replay; the ranks pace each other through the inbox flags, so the
    host only enqueues replays.  Message layouts come from the first (eager, packed)
    step's signatures, identical at both ends."""

    def __init__(self, plan, rank, link, meta, dev, key):
        from .hop import BulkInbox, BulkPeer
        self.rank, self.dev, self.meta = rank, dev, meta
        self.inbox: dict = {}
        self.state: dict = {}
        self.views: dict = {}
        self.peers: dict = {}
        self.out_layout: dict = {}
        mine = {}
        err = None
        try:
            for a, items in plan.incoming(rank):
                dt, shapes = link._recv[(a, key(a, rank))]
                esz = torch.empty((), dtype=_DT[dt]).element_size()
                sizes = [int(torch.Size(sh).numel()) * esz for sh in shapes]
                offs, cap = _layout(sizes)
                box = BulkInbox(cap, dev)
                buf = torch.empty(box.nbytes, dtype=torch.uint8, device=dev)
                self.inbox[a], self.state[a] = box, buf
                self.views[a] = {it: buf[o:o + n].view(_DT[dt]).view(sh)
                                 for it, o, n, sh in zip(items, offs, sizes, shapes)}
                mine[(a, rank)] = (box.handle(), box.nbytes)
            for b, items in plan.outgoing(rank):
                dt, shapes = link._sent[(b, key(rank, b))]
                esz = torch.empty((), dtype=_DT[dt]).element_size()
                sizes = [int(torch.Size(sh).numel()) * esz for sh in shapes]
                self.out_layout[b] = _layout(sizes)
        except Exception as e:  # noqa: BLE001  (every rank learns of it below)
            err = f"rank {rank}: {type(e).__name__}: {e}"[:300]
        allh: list = [None] * dist.get_world_size(meta)
        dist.all_gather_object(allh, (mine, err), group=meta)
        bad = [e for _, e in allh if e]
        if bad:
            raise RuntimeError("split-UNet device hops: " + "; ".join(bad))
        handles = {}
        for m, _ in allh:
            handles.update(m)
        for b, _ in plan.outgoing(rank):
            h, cap = handles[(rank, b)]
            if cap != (self.out_layout[b][1] + 15) // 16 * 16:
                raise RuntimeError(f"split-UNet channel {rank}->{b}: layouts disagree "
                                   f"({cap} vs {self.out_layout[b][1]} bytes)")
            self.peers[b] = BulkPeer(h, cap, dev)

    def bytes_per_channel(self) -> dict:
        return {f"{self.rank}->{b}": lay[1] for b, lay in self.out_layout.items()}

    def recv(self, a):
        self.inbox[a].recv(self.state[a])
        return dict(self.views[a])

    def send(self, b, items, tensors):
        ts = [t if t.is_contiguous() else t.contiguous() for t in tensors]
        self.peers[b].send(ts, self.out_layout[b][0])

    def run(self, plan, rank, world, my_run, run_stages, inp, after, step_dev, n: int,
            warm: int):
        """Capture this rank's step graph, time its compute alone (a compute-only graph,
        ranks one after another), then replay the step n times in lock step with the
        other ranks; rank 0's per-step times of the last n - warm replays."""
        from ..ops import hip as K

        def body():
            if my_run is not None:
                pred = plan.step(rank, inp if rank == 0 else None, run_stages, self.recv,
                                 self.send)
                if rank == 0:
                    after(pred)
            K.step_advance(step_dev)

        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            body()
        compute: list[float] = []
        if my_run is not None:
            xin = inp if rank == plan.order[0] else None
            got: dict = {}
            for a, _ in plan.incoming(rank) if rank != plan.order[0] else []:
                got.update(self.views[a])
            if xin is None:
                xin = got.pop("x")
            skips = [got[i] for i in plan.received_skips(rank)]
            gc = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gc, stream=s):
                run_stages(xin, list(skips))
            # the time bias index is read at replay: keep it in range
            saved = step_dev.clone()
            for r in range(world):
                if r == rank:
                    for _ in range(3):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record()
                        gc.replay()
                        e1.record()
                        e1.synchronize()
                        compute.append(e0.elapsed_time(e1) / 1e3)
                dist.barrier()
            step_dev.copy_(saved)
            del gc
        else:
            for _ in range(world):
                dist.barrier()
        torch.cuda.synchronize(self.dev)
        dist.barrier()
        evs = []
        for i in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            graph.replay()
            e1.record()
            if i >= warm:
                evs.append((e0, e1))
        torch.cuda.synchronize(self.dev)
        errs = [a for a, box in self.inbox.items() if box.error()]
        bad: list = [None] * world
        dist.all_gather_object(bad, errs, group=self.meta)
        if any(bad):
            raise RuntimeError("split-UNet device hop receive timed out: " +
                               ", ".join(f"rank {r} from {e}" for r, e in enumerate(bad) if e))
        del graph
        return [a.elapsed_time(b) / 1e3 for a, b in evs], compute

    def close(self, meta) -> None:
        for p in self.peers.values():
            p.close()
        dist.barrier(group=meta)  # every importer unmapped before the inboxes go
        for b in self.inbox.values():
            b.close()
