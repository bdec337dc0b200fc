"""Master/worker roles over RCCL (``--transport rccl``, launched with torchrun).

One process per GPU of a node: rank 0 is the master (tokenizer, embedding,
ln_f, lm_head, sampling, CLI or REST API, plus every layer no worker owns);
rank i >= 1 serves the i-th node of ``topology.yml`` (file order).  Hidden
states hop device-to-device (``parallel/pipeline.py``) instead of cake's TCP
frames (cake-core/src/cake/client.rs:116-124, worker.rs:236-252): by default
as device-side peer stores captured in every rank's decode graph (``--hop
ipc``; host-issued RCCL p2p with ``--hop dist`` or when the IPC self-test
fails), with every request announced to the workers on a host control channel
(``PipelineEngine.serve``).  Each rank loads only the tensors it owns from the
checkpoint (or a split-model bundle).

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m cake_amd.cli \\
        --transport rccl --model M --topology topology.yml --api 0.0.0.0:8080
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

from ..models.base import TextGenerator, Token
from ..models.chat import History
from ..models.sampling import LogitsProcessor
from .pipeline import PipelineEngine, init_process_group

log = logging.getLogger("cake.rccl")


def owners_from_topology(topology, num_layers: int, world: int) -> list[int]:
    owners = [0] * num_layers
    if len(topology.nodes) > world - 1:
        raise ValueError(f"topology has {len(topology.nodes)} workers but only {world - 1} "
                         "worker ranks were launched")
    for i, node in enumerate(topology.nodes):
        for name in node.layers:
            if name.startswith("model.layers."):
                li = int(name.split(".")[-1])
                if 0 <= li < num_layers:
                    owners[li] = i + 1
    return owners


class PipelineLLM(TextGenerator):
    """TextGenerator over the RCCL pipeline (master rank)."""
    MODEL_NAME = "llama3"

    def __init__(self, engine: PipelineEngine, tokenizer, eos_ids, sampling):
        self.eng, self.tokenizer, self.eos_ids, self.sampling = engine, tokenizer, set(eos_ids), sampling
        self.history = History()
        self.tokens: list[int] = []
        self.generated = 0
        if not sampling.greedy:
            if engine.hip:   # seeded temperature / top-k / top-p draw inside the graph
                engine.sampling = sampling
            else:
                engine.sampler = LogitsProcessor(sampling).sample
        self.last_stats = None

    @classmethod
    def load(cls, ctx):
        """Master-rank generator of an already running RCCL job (run_rccl builds the
        engine collectively on every rank first; ``ctx.engine`` is that engine)."""
        from ..models.llama3.generator import load_tokenizer
        eng = getattr(ctx, "engine", None)
        if eng is None or not eng.is_master:
            raise RuntimeError("PipelineLLM.load needs ctx.engine: the master rank's "
                               "PipelineEngine (see run_rccl)")
        tok, eos = load_tokenizer(ctx.model_path, eng.cfg.eos_token_id)
        return cls(eng, tok, eos, ctx.sampling)

    def metrics(self) -> dict:
        """--metrics fields of the pipeline: hop latency measured at start-up
        (µs, device-timed ping-pong), hops per token, and every rank's HBM."""
        return dict(getattr(self.eng, "metrics", {}) or {})

    def set_sampling(self, sampling) -> None:
        self.sampling = sampling
        self.eng.set_sampling(sampling)

    def add_message(self, message) -> None:
        self.history.append(message)

    def reset(self) -> None:
        self.history.clear()
        self.tokens.clear()
        self.generated = 0

    def generated_tokens(self) -> int:
        return self.generated

    def _token(self, tid: int) -> Token:
        self.generated += 1
        self.tokens.append(tid)
        return Token(tid, self.tokenizer.decode([tid], skip_special_tokens=False),
                     tid in self.eos_ids)

    def _prefill(self) -> int:
        self.tokens = self.tokenizer.encode(self.history.encode_dialog_to_prompt(),
                                            add_special_tokens=False).ids
        self.eng.ctrl_send({"op": "prefill"})
        return self.eng.prefill(0, self.tokens)

    def next_token(self, index: int) -> Token:
        if self.generated == 0:
            return self._token(self._prefill())
        got = self.eng.generate(1)
        if not got:
            raise RuntimeError("KV cache full (--max-seq-len)")
        return self._token(got[0])

    def stream(self, max_tokens, on_token, stop_at_eos=True):
        """Prefill, then up to max_tokens - 1 decode tokens through the pipeline in
        control-announced chunks (clamped to the KV cache), stopping at EOS."""
        out = []
        if max_tokens <= 0:
            return out
        t = self._token(self._prefill())
        out.append(t)
        on_token(t)
        if t.is_end_of_stream and stop_at_eos:
            return out

        def cb(tid: int) -> None:
            tk = self._token(tid)
            out.append(tk)
            on_token(tk)
        self.eng.generate(max_tokens - 1, cb, self.eos_ids if stop_at_eos else None)
        return out


class TPLLM(TextGenerator):
    """TextGenerator over the tensor-parallel engine (rank 0).  Every generation is a
    broadcast command the other ranks execute in lock step (``_tp_follow``); all
    ranks see the same tokens, so each detects EOS by itself."""
    MODEL_NAME = "llama3"

    def __init__(self, eng, tokenizer, eos_ids, sampling):
        self.eng, self.tokenizer, self.eos_ids = eng, tokenizer, set(eos_ids)
        self.sampling = sampling
        self.history = History()
        self.generated = 0
        self.last_stats = None

    @classmethod
    def load(cls, ctx):
        """Rank-0 generator of a running TP job (``ctx.engine``: its TPEngine)."""
        from ..models.llama3.generator import load_tokenizer
        eng = getattr(ctx, "engine", None)
        if eng is None or eng.rank != 0:
            raise RuntimeError("TPLLM.load needs ctx.engine: rank 0's TPEngine (see run_tp)")
        tok, eos = load_tokenizer(ctx.model_path, eng.cfg.eos_token_id)
        return cls(eng, tok, eos, ctx.sampling)

    def add_message(self, message) -> None:
        self.history.append(message)

    def reset(self) -> None:
        self.history.clear()
        self.generated = 0

    def generated_tokens(self) -> int:
        return self.generated

    def set_sampling(self, sampling) -> None:
        """Per-request sampling: temperature / top_k / top_p / seed all travel in the
        generate command; the ranks rewrite their device parameter blocks (no
        recapture)."""
        self.sampling = sampling

    def next_token(self, index: int) -> Token:  # pragma: no cover - stream() drives it
        raise NotImplementedError("use stream()")

    def stream(self, max_tokens, on_token, stop_at_eos=True):
        prompt = self.tokenizer.encode(self.history.encode_dialog_to_prompt(),
                                       add_special_tokens=False).ids
        s = self.sampling
        cmd = {"op": "generate", "prompt": prompt, "max_tokens": int(max_tokens),
               "eos": sorted(self.eos_ids) if stop_at_eos else [],
               "temperature": 0.0 if s.greedy else float(s.temperature), "seed": int(s.seed),
               "top_k": int(s.top_k or 0), "top_p": float(s.top_p) if s.top_p is not None else None}
        dist.broadcast_object_list([cmd], src=0)
        out = []

        def emit(tid):
            self.generated += 1
            t = Token(tid, self.tokenizer.decode([tid], skip_special_tokens=False),
                      tid in self.eos_ids)
            out.append(t)
            on_token(t)
        self.last_stats = _tp_generate(self.eng, cmd, emit)
        return out


def _tp_generate(eng, cmd, emit=None):
    """One generation on every rank (same command, same tokens).  The sampling
    configuration goes to the device parameter block (no recapture when only the
    temperature / seed / top-k / top-p change); tokens are read back one step
    behind the GPU (the next step is enqueued before the previous token is read),
    and every rank stops after the same token."""
    from ..models.llama3.decode_loop import DecodeStats
    from ..models.sampling import SamplingConfig
    temp = float(cmd["temperature"])
    eng.set_sampling(None if temp <= 0 else SamplingConfig(
        temperature=temp, top_k=int(cmd.get("top_k") or 0) or None, top_p=cmd.get("top_p"),
        seed=int(cmd["seed"]), repeat_penalty=eng.penalty, repeat_last_n=eng.last_n))
    # the first token comes from the prefill; every later one needs a cache row
    n = min(int(cmd["max_tokens"]), eng.max_seq - len(cmd["prompt"]))
    eos = set(cmd["eos"])
    st = DecodeStats()
    if n <= 0:
        return st
    tid = eng.prefill(cmd["prompt"])
    eng.capture()
    if emit is not None:
        emit(tid)
    if tid in eos or n == 1:
        eng.check()
        return st
    if not eng.hip:
        for _ in range(n - 1):
            tid = eng.step()
            if emit is not None:
                emit(tid)
            if tid in eos:
                break
        eng.check()
        return st
    b = eng.b
    base = int(b.hist_len.item())
    if eng.use_graph and eng.mode in eng.graphs:
        # native decode driver (csrc/driver/graph_loop.cpp): every rank replays and
        # reads back the same tokens, so all stop after the same one
        from ..ops import graph_loop as GL
        # the callback (rank 0 only) must not change this rank's replay count: every
        # rank stops at the same EOS, whatever the callback returns or raises
        res = GL.run(eng.graph_set(), k=1, n=n - 1, pos=eng.host_pos, hist=b.hist, base=base,
                     eos_ids=eos, on_token=(lambda t: bool(emit(t))) if emit is not None
                     else None, callback_stops=False)
        eng.host_pos = res.pos
        st.tokens, st.step_ms, st.wall_s = res.tokens, res.step_ms, res.wall_s
        eng.tokens = b.hist[:int(b.hist_len.item())].tolist()
        eng.check()
        return st
    ring = torch.empty(n, dtype=torch.int32, pin_memory=True)
    prev = torch.cuda.Event(enable_timing=True)
    prev.record()
    pending = None
    for i in range(n - 1):
        eng.launch()
        ring[i:i + 1].copy_(b.hist[base + i:base + i + 1], non_blocking=True)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        cur = (i, ev)
        if pending is not None and _tp_take(eng, pending, ring, prev, st, emit, eos):
            pending = None
            break
        if pending is not None:
            prev = pending[1]
        pending = cur
    if pending is not None:
        _tp_take(eng, pending, ring, prev, st, emit, eos)
    torch.cuda.synchronize(eng.device)
    eng.tokens = b.hist[:int(b.hist_len.item())].tolist()
    eng.check()
    return st


def _tp_take(eng, pending, ring, prev, st, emit, eos) -> bool:
    """Read one enqueued step's token; True at EOS."""
    i, ev = pending
    ev.synchronize()
    tid = int(ring[i].item())
    st.step_ms.append(prev.elapsed_time(ev))
    st.tokens.append(tid)
    if emit is not None:
        emit(tid)
    return tid in eos


def _tp_follow(eng) -> None:
    """Ranks >= 1 of a tensor-parallel job: execute rank 0's commands until "stop"."""
    while True:
        box = [None]
        dist.broadcast_object_list(box, src=0)
        cmd = box[0]
        if cmd is None or cmd.get("op") == "stop":
            return
        _tp_generate(eng, cmd)


def _init_dist(ctx, rank: int, world: int) -> None:
    """One rank per GPU (LOCAL_RANK); RCCL ("nccl") on GPUs, gloo on the CPU.
    CAKE_DIST_BACKEND=gloo lets several ranks share one GPU (RCCL refuses duplicate
    devices): tests and single-GPU rehearsals; decode hops stay device-side (ipc)."""
    backend = os.environ.get("CAKE_DIST_BACKEND")
    if ctx.device.type == "cuda":
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        ctx.device = torch.device("cuda", local)
        backend = backend or "nccl"
        init_process_group(backend, rank, world, ctx.device)
    else:
        init_process_group("gloo", rank, world)


def run_tp(ctx) -> None:
    """``--transport rccl --parallel tp``: every rank loads 1/N of every layer (the
    topology's layer placement does not apply); rank 0 runs the master / API."""
    from ..models.llama3.config import LlamaConfig
    from .tensor_parallel import AllReduce, TPEngine, check_tp, load_shards
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    _init_dist(ctx, rank, world)
    try:
        cfg = LlamaConfig.from_path(ctx.model_path)
        check_tp(cfg, world)
        blocks, head = load_shards(ctx.model_path, cfg, rank, world, ctx.device, ctx.dtype)
        comm = AllReduce(rank, world, ctx.device, cfg.hidden_size, n_gather=cfg.vocab_size,
                         mode=getattr(ctx.args, "allreduce", "ipc"))
        s = ctx.sampling
        eng = TPEngine(cfg, blocks, head, rank, world, ctx.device, ctx.dtype, ctx.max_seq_len,
                       comm, repeat_penalty=s.repeat_penalty, repeat_last_n=s.repeat_last_n,
                       use_graph=not ctx.no_graph)
        log.info("rank %d/%d: tensor-parallel shard, all-reduce %s", rank, world, comm.mode)
        if rank == 0:
            from ..master import Master
            ctx.engine = eng
            llm = TPLLM.load(ctx)
            llm.set_sampling(s)
            try:
                Master(ctx, llm=llm).run()
            finally:
                dist.broadcast_object_list([{"op": "stop"}], src=0)
        else:
            _tp_follow(eng)
        comm.close()
    finally:
        dist.destroy_process_group()


def _native_rank_engine(ctx, rank: int, world: int, tp: bool):
    """This rank's native engine of the group (pp: the topology's placement; tp: 1/N of
    every layer).  Its control plane listens on MASTER_PORT + 1 (torchrun's store owns
    MASTER_PORT); the decode hops / all-reduces are device-side inside every rank's graph."""
    from ..engine import NativeLlama
    from ..models.llama3.config import LlamaConfig
    from ..models.llama3.native_generator import _dtype_name
    a = ctx.args
    cfg = LlamaConfig.from_path(ctx.model_path)
    owners = None if tp else owners_from_topology(ctx.topology, cfg.num_hidden_layers, world)
    if owners is not None and not any(owners):
        owners = None  # no node places a layer: contiguous shards
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    addr = f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{int(os.environ.get('MASTER_PORT', '29500')) + 1}"
    timeout = float(os.environ.get("CAKE_HOP_TIMEOUT", "60"))
    return NativeLlama(ctx.model_path, max_seq=ctx.max_seq_len, dtype=_dtype_name(ctx.dtype),
                       device=local, rank=rank, world=world, master_addr=addr,
                       hop_bf16=getattr(a, "hop_dtype", "f32") == "bf16", hop_timeout_s=timeout,
                       tp=tp, owners=owners)


def _native_group(ctx) -> bool:
    """--transport rccl on the native engine: a GPU, 16-bit weights, graphs, device hops
    (--hop ipc) or tensor parallel; CAKE_NATIVE=0 keeps the Python engines."""
    from ..models.llama3.native_generator import native_eligible
    a = ctx.args
    tp = getattr(a, "parallel", "pp") == "tp"
    return native_eligible(ctx) and (tp or getattr(a, "hop", "ipc") == "ipc")


def run_native_rccl(ctx) -> bool:
    """Every rank runs the native engine; rank 0 is the master (CLI generation or the
    REST API over :class:`NativeLLM`), the others serve it until it closes.  False (and
    nothing served) when the engine's start-up self-test refused the device transport."""
    from ..models.llama3.native_generator import NativeLLM
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    tp = getattr(ctx.args, "parallel", "pp") == "tp"
    if ctx.device.type == "cuda":
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
    try:
        eng = _native_rank_engine(ctx, rank, world, tp)
    except RuntimeError as e:
        if "self-test failed" not in str(e):
            raise
        # the group's device IPC transport failed its start-up self-test (the verdict
        # reaches every rank): all ranks run the Python engines over RCCL instead
        log.warning("rank %d/%d: native engine refused the device transport (%s); "
                    "serving over torch.distributed (RCCL) instead", rank, world, e)
        return False
    log.info("rank %d/%d: native engine, %s", rank, world,
             "tensor parallel" if tp else f"walk {eng.walk()} (hops: ipc)")
    try:
        if rank == 0:
            from ..master import Master
            Master(ctx, llm=NativeLLM.load(ctx, engine=eng)).run()
        else:
            eng.serve()
    finally:
        eng.close()
    return True


def run_rccl(ctx) -> None:
    if ctx.model_type == "image-model":
        from .sd_rccl import run_sd_rccl
        run_sd_rccl(ctx)
        return
    if _native_group(ctx):
        if run_native_rccl(ctx):
            return
        ctx.args.hop = "dist"  # the fallback transport: RCCL p2p / all-reduce
        ctx.args.allreduce = "dist"
    if getattr(ctx.args, "parallel", "pp") == "tp":
        run_tp(ctx)
        return
    from ..models.llama3.config import LlamaConfig
    from ..models.llama3.factory import load_stack
    from ..models.llama3.generator import load_tokenizer
    from ..models.llama3.weights import HeadWeights
    from ..utils.safetensors_io import ShardedCheckpoint

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    _init_dist(ctx, rank, world)
    try:
        cfg = LlamaConfig.from_path(ctx.model_path)
        owners = owners_from_topology(ctx.topology, cfg.num_hidden_layers, world)
        mine = [li for li, r in enumerate(owners) if r == rank]
        stack = load_stack(ctx.model_path, cfg, mine, ctx.device, ctx.dtype, ctx.max_seq_len)
        head = None
        if rank == 0:
            head = HeadWeights.load(ShardedCheckpoint(ctx.model_path).get, cfg, ctx.device, ctx.dtype)
        s = ctx.sampling
        a = ctx.args
        eng = PipelineEngine(cfg, stack, owners, rank, world, streams=1, head=head,
                             repeat_penalty=s.repeat_penalty, repeat_last_n=s.repeat_last_n,
                             use_graph=not ctx.no_graph, hop=getattr(a, "hop", "ipc"),
                             hop_bf16=getattr(a, "hop_dtype", "f32") == "bf16")
        log.info("rank %d/%d owns layers %s (hops: %s)", rank, world,
                 mine[:3] + (["..."] if len(mine) > 3 else []), eng.hop)
        if rank == 0 and eng.hip:
            eng.set_sampling(s)  # device-read parameters: per-request API sampling
        if eng.use_graph:
            # the graphs read the position from device state; a dummy prefill gives
            # every graph valid state to capture against (collective, at start-up)
            eng.prefill(0, [cfg.bos_token_id or 0] if rank == 0 else None)
            eng.flush()
            eng.capture()
        _startup_metrics(eng, ctx, rank, world, len(mine))
        if rank == 0:
            from ..master import Master
            ctx.engine = eng
            master = Master(ctx, llm=PipelineLLM.load(ctx))
            try:
                master.run()
            finally:
                eng.shutdown()
        else:
            eng.serve()
        eng.close()
    finally:
        dist.destroy_process_group()


def _startup_metrics(eng: PipelineEngine, ctx, rank: int, world: int, n_layers: int) -> None:
    """Collective, once: per-hop latency (rank 0 <-> 1 ping-pong over the configured
    transport) and each rank's HBM / layer count, kept on the master's engine."""
    from ..context import hbm_mib
    hop_us = eng.measure_hop_us() if world > 1 else None
    mine = {"rank": rank, "layers": n_layers,
            **(hbm_mib(ctx.device) if ctx.device.type == "cuda" else {})}
    ranks = [None] * world
    dist.all_gather_object(ranks, mine)
    hops = eng.hops_per_token()
    eng.metrics = {"hop_us": None if hop_us is None else round(hop_us, 2),
                   "hops_per_token": hops, "rank_hbm": ranks}
    if rank == 0:
        log.info("pipeline: %d hops/token, hop %s us; per-rank HBM %s", hops,
                 "n/a" if hop_us is None else f"{hop_us:.1f}",
                 [r.get("hbm_used_mib") for r in ranks])
