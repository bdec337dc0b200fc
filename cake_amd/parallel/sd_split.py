"""Split-UNet diffusion over N ranks: BASELINE config 5 ("SDXL UNet blocks sharded
across workers") as a measured path.

The reference reaches a remote UNet once per diffusion step — the latents, text
embedding and timestep packed into one f32 buffer and copied device -> host ->
socket -> host -> device each way (cake-core/src/models/sd/sd.rs:464-513, the
per-step time including that round trip at :506-507; unet.rs:81-100 packing;
sd_shardable.rs:29-45 dispatch).  Here the UNet's block groups (``down.i``,
``mid``, ``up.i``: UNet2DConditionModel.stage_names) are spread over the ranks
contiguously, and one diffusion step walks them in order: the running feature map
and the skip stack of the down path move rank to rank as ONE packed device buffer
per hop over RCCL (xGMI), device to device, issued on the compute stream with no
per-step host metadata (:class:`PackedLink`: shapes are exchanged once, on the first
hop of a signature).  The text embedding reaches each stage owner once; the
cross-attention k/v of it are cached there for every step.  Rank 0 (the master)
owns the first stages and the CFG combine + scheduler update.
"""
from __future__ import annotations

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
    nxt = runs[my_run + 1][0] if my_run is not None and my_run < last else 0
    prv = runs[my_run - 1][0] if my_run is not None and my_run > 0 else None
    inp = torch.empty(2, *lat.shape[1:], device=dev, dtype=dtype)
    x = lat.clone() * sched.init_noise_sigma
    step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
    seed_dev = torch.zeros(1, dtype=torch.int64, device=dev)
    coef_dev = coef.to(dev)
    compute_s: list[float] = []
    step_s: list[float] = []

    def sync():
        if hip:
            torch.cuda.synchronize(dev)

    dist.barrier()
    for i, t in enumerate(ts):
        sync()
        t0 = time.perf_counter()
        if rank == 0:
            if hip:
                from ..ops import hip as K
                K.scale_copy(x, sched.input_scale(t), True, inp)
            else:
                inp.copy_((x * sched.input_scale(t)).expand(2, -1, -1, -1))
            state = [inp]
        elif my_run is not None:
            state = link.recv(prv, "unet")
        if my_run is not None:
            sync()
            c0 = time.perf_counter()
            xs, skips = model.forward_stages(W, names, state[0], list(state[1:]), float(t), emb,
                                             kv_cache=kv)
            sync()
            if i >= warmup:
                compute_s.append(time.perf_counter() - c0)
            if my_run == last:
                if last > 0:  # (one rank: the master already holds the output)
                    link.send([xs], 0, "unet_out")
            else:
                link.send([xs] + skips, nxt, "unet")
        if rank == 0:
            pred = link.recv(runs[last][0], "unet_out")[0] if last > 0 else xs
            if hip:
                K.sched_step(x, pred, True, 7.5, coef_dev, step_dev, seed_dev)
                K.step_advance(step_dev)
            else:
                x = _sched_update(x, pred, coef[i], 7.5)
            sync()
            if i >= warmup:
                step_s.append(time.perf_counter() - t0)
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
    hops = len(runs)  # runs - 1 forward hops + the output back to the master
    comp_sum = sum(comp)
    return {"seconds_per_step": round(per_step, 5), "version": version,
            "resolution": f"{cfg.width}x{cfg.height}", "batch": 2,
            "dtype": {torch.float16: "f16", torch.bfloat16: "bf16",
                      torch.float32: "f32"}[dtype],
            "ranks_used": len(runs), "stages": {f"rank{r}": n for r, n in runs},
            "compute_s_per_rank": [round(c, 5) for c in comp],
            "hops_per_step": hops,
            "hop_us_mean": round(max(0.0, per_step - comp_sum) / hops * 1e6, 1) if hops else 0.0,
            "steps": steps, "warmup": warmup,
            "per_step_s": [round(s, 5) for s in step_s],
            # the final latents (equivalence across rank counts; tests)
            "latent_checksum": float(x.double().sum()), "latent_abs": float(x.double().abs().sum()),
            "transport": ("gloo, host-staged packed buffer per hop" if link.staged else
                          "rccl p2p, packed buffer per hop") if hip else "gloo"}
