"""Tensor-parallel batch-1 decode over the GPUs of one node (MI355X-first mode).

The reference scales a model over workers by sharding LAYERS
(cake-core/src/models/llama3/llama.rs:95-114, topology.yml): a token visits
every worker in turn, so N GPUs decode one sequence no faster than one GPU
(``parallel/pipeline.py`` keeps that mode, with graph-resident hops).  Batch-1
decode is HBM-bound, so here every rank instead holds 1/N of EVERY layer —
its share of the attention heads (q rows of its heads, the matching K/V heads,
the o_proj columns) and of the MLP (gate/up rows, down_proj columns) — and
streams 1/N of the weights per token.  Two all-reduces of the hidden state per
layer (after o_proj, after down_proj) and one argmax-key max over the
vocabulary-sharded lm_head make the ranks agree; on the HIP path they are
``allreduce.hip`` one-shot kernels over xGMI captured in each rank's decode
graph (RCCL / ``torch.distributed`` as the fallback and for prefill).

Every rank keeps the full embedding table, so all ranks embed the selected
token locally and stay in lock step with no broadcast.  Token selection:
greedy (with the reference's repeat penalty) = shard argmax key + one 64-bit
max all-reduce; sampled (temperature / top-k / top-p, the reference's
LogitsProcessor, cake-core/src/models/llama3/llama.rs:34-48, 323-326) = the
vocabulary shards are all-gathered into a full logits vector on every rank
(allreduce.hip ar_gather, device-side), then every rank runs the single-GPU
device selection (repeat penalty, top-k/top-p threshold, Philox Gumbel-max
keyed by the GLOBAL index) on identical inputs and picks the same token — equal
to the single-GPU draw.  The sampling configuration lives in a device
parameter block, so a request with another temperature / seed / top-k / top-p
replays the same graphs (one graph set per greedy/sampled mode).

Shards: ``shard_block`` / ``shard_head`` cut a full checkpoint's tensors
(heads and MLP rows split contiguously: rank r owns q heads
[r·nh/N, (r+1)·nh/N) and therefore KV heads [r·nkv/N, ...) of a GQA model);
``random_shards`` builds random-init shards of the right shapes directly
(benchmarks: no full model on any rank).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import logging
import math
import os

import torch
import torch.distributed as dist

from ..models.llama3.config import LlamaConfig
from ..models.llama3.weights import BlockWeights
from ..ops import reference as R

log = logging.getLogger("cake.tp")


def split_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """[start, end) of rank's contiguous share of n items (sizes differ by <= 1)."""
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def check_tp(cfg: LlamaConfig, world: int) -> None:
    nh, nkv = cfg.num_attention_heads, cfg.num_key_value_heads
    if world < 1 or nkv % world or nh % world:
        raise ValueError(f"tensor parallel degree {world} must divide the {nkv} KV heads "
                         f"and {nh} query heads")


@dataclasses.dataclass
class TPHead:
    embed: torch.Tensor   # [V, H] full table (every rank embeds the selected token)
    norm: torch.Tensor    # [H]
    lm: torch.Tensor      # [V_r, H] rows [voff, voff + V_r) of lm_head
    voff: int


def shard_block(w: BlockWeights, cfg: LlamaConfig, rank: int, world: int, device=None,
                dtype=None) -> BlockWeights:
    """This rank's slice of one full decoder block."""
    check_tp(cfg, world)
    hd = cfg.head_dim
    q0, q1 = split_range(cfg.num_attention_heads, world, rank)
    k0, k1 = split_range(cfg.num_key_value_heads, world, rank)
    i0, i1 = split_range(cfg.intermediate_size, world, rank)

    def t(x):
        return x.to(device or x.device, dtype or x.dtype).contiguous()
    return BlockWeights(ln1=t(w.ln1), wq=t(w.wq[q0 * hd:q1 * hd]), wk=t(w.wk[k0 * hd:k1 * hd]),
                        wv=t(w.wv[k0 * hd:k1 * hd]), wo=t(w.wo[:, q0 * hd:q1 * hd]),
                        ln2=t(w.ln2), wg=t(w.wg[i0:i1]), wu=t(w.wu[i0:i1]), wd=t(w.wd[:, i0:i1]))


def shard_head(embed, norm, lm_head, rank: int, world: int, device=None, dtype=None) -> TPHead:
    v0, v1 = split_range(lm_head.shape[0], world, rank)

    def t(x):
        return x.to(device or x.device, dtype or x.dtype).contiguous()
    return TPHead(embed=t(embed), norm=t(norm), lm=t(lm_head[v0:v1]), voff=v0)


def random_shards(cfg: LlamaConfig, rank: int, world: int, device, dtype, seed: int = 0,
                  layers: list[int] | None = None) -> tuple[dict, TPHead]:
    """Random-init shards of this rank's shapes (std 0.02 like the synthetic models);
    the embedding and norms come from the same seed on every rank."""
    check_tp(cfg, world)
    H, hd = cfg.hidden_size, cfg.head_dim
    q0, q1 = split_range(cfg.num_attention_heads, world, rank)
    k0, k1 = split_range(cfg.num_key_value_heads, world, rank)
    i0, i1 = split_range(cfg.intermediate_size, world, rank)
    v0, v1 = split_range(cfg.vocab_size, world, rank)
    gen = torch.Generator(device=device).manual_seed(seed * 1000003 + rank)
    shared = torch.Generator(device=device).manual_seed(seed)

    def rnd(*shape, std=0.02, g=gen):
        return torch.empty(shape, device=device, dtype=dtype).normal_(0.0, std, generator=g)

    def ones(n):
        return torch.empty((n,), device=device, dtype=dtype).normal_(1.0, 0.05, generator=shared)
    blocks = {}
    for li in (layers if layers is not None else range(cfg.num_hidden_layers)):
        blocks[li] = BlockWeights(ln1=ones(H), wq=rnd((q1 - q0) * hd, H), wk=rnd((k1 - k0) * hd, H),
                                  wv=rnd((k1 - k0) * hd, H), wo=rnd(H, (q1 - q0) * hd),
                                  ln2=ones(H), wg=rnd(i1 - i0, H), wu=rnd(i1 - i0, H),
                                  wd=rnd(H, i1 - i0))
    embed = rnd(cfg.vocab_size, H, std=1.0, g=shared)
    head = TPHead(embed=embed, norm=ones(H), lm=rnd(v1 - v0, H), voff=v0)
    return blocks, head


def load_shards(model_path: str, cfg: LlamaConfig, rank: int, world: int, device,
                dtype) -> tuple[dict, TPHead]:
    """This rank's shards of a Hugging Face checkpoint (only the slices are copied)."""
    from ..utils.safetensors_io import ShardedCheckpoint
    from ..models.llama3.weights import HeadWeights
    ck = ShardedCheckpoint(model_path)
    blocks = {}
    for li in range(cfg.num_hidden_layers):
        full = BlockWeights.load(ck.get, f"model.layers.{li}", cfg, "cpu", dtype)
        blocks[li] = shard_block(full, cfg, rank, world, device, dtype)
    hw = HeadWeights.load(ck.get, cfg, "cpu", dtype)
    return blocks, shard_head(hw.embed, hw.norm, hw.lm_head, rank, world, device, dtype)


# ---------------------------------------------------------------------------
# all-reduce channels
# ---------------------------------------------------------------------------
class AllReduce:
    """Sum of f32 vectors and max of the u64 argmax key over the TP group.

    mode "ipc": allreduce.hip one-shot kernels (device-side, graph-capturable), two
    channels (hidden-size sums, 2-word keys), each with its own inbox (uncached,
    IPC-exported) and tag counter; a start-up self-test must pass on every rank or
    the group falls back to "dist" (torch.distributed, RCCL on GPUs / gloo)."""

    def __init__(self, rank: int, world: int, device, n: int, mode: str = "ipc", group=None,
                 n_gather: int = 0):
        self.rank, self.world, self.device, self.n = rank, world, torch.device(device), n
        self.n_gather = int(n_gather)  # gather channel width (vocabulary; 0 = none)
        self.group = group
        self.mode = mode if (world > 1 and self.device.type == "cuda") else "dist"
        self.staged = (world > 1 and dist.is_initialized()
                       and dist.get_backend(group) == "gloo")
        self._inboxes, self._peers = [], []
        self.gather_ch = None
        self.timeout_s = float(os.environ.get("CAKE_HOP_TIMEOUT", "60"))
        if self.mode == "ipc":
            # every rank runs the same collective sequence whatever fails locally
            # (one handle exchange, one self-test, one agreement), so a failure on
            # one rank falls back instead of leaving the others in a collective
            ok = self._setup_ipc()
            if ok:
                try:
                    ok = self._selftest()
                except Exception as e:  # noqa: BLE001  (agreed on below)
                    log.warning("tp all-reduce IPC self-test failed on rank %d: %s", rank, e)
                    ok = False
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
            self._all_reduce_host(flag, dist.ReduceOp.MIN)
            if int(flag.item()) != 1:
                if rank == 0:
                    log.warning("tp all-reduce: IPC self-test failed -> torch.distributed")
                self._close_ipc()
                self.mode = "dist"

    # -- host-side collectives (setup, fallback, prefill)
    def _all_reduce_host(self, t: torch.Tensor, op=None) -> None:
        op = op if op is not None else dist.ReduceOp.SUM
        if dist.get_backend(self.group) == "gloo":
            dist.all_reduce(t, op=op, group=self.group)
        else:
            d = t.to(self.device)
            dist.all_reduce(d, op=op, group=self.group)
            t.copy_(d.cpu())

    def dense_sum_(self, t: torch.Tensor) -> None:
        """In-place sum of any tensor over the group (prefill: [T, H] partials)."""
        if self.world == 1:
            return
        if self.staged and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)

    # -- IPC channels
    def _setup_ipc(self) -> bool:
        """Both channels' inboxes, ONE handle exchange (joined even after a local
        failure, with None handles), then the peer mappings.  The self-test runs only
        if every rank mapped every peer (agreed with a MIN); returns that agreement."""
        from .hop import Inbox, PeerInbox
        sizes = {"sum": 2 * self.world * self.n, "key": 2 * self.world * 2}  # inbox granules
        if self.n_gather:
            sizes["gather"] = 2 * self.n_gather
        mine = None
        try:
            ibs = {k: Inbox(n) for k, n in sizes.items()}
            self._inboxes.extend(ibs.values())
            mine = {k: ib.handle() for k, ib in ibs.items()}
        except Exception as e:  # noqa: BLE001
            log.warning("tp all-reduce inbox allocation failed on rank %d: %s", self.rank, e)
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=self.group)
        ok = all(h is not None for h in handles)
        chans = {}
        if ok:
            try:
                for k in sizes:
                    peers = (C.c_void_p * 8)()
                    for r in range(self.world):
                        if r != self.rank:
                            p = PeerInbox(handles[r][k])
                            self._peers.append(p)
                            peers[r] = p.ptr
                    chans[k] = {"inbox": ibs[k], "peers": peers,
                                "seq": torch.zeros(2, dtype=torch.int32, device=self.device),
                                "err": torch.zeros(1, dtype=torch.int32, device=self.device)}
            except Exception as e:  # noqa: BLE001
                log.warning("tp all-reduce IPC open failed on rank %d: %s", self.rank, e)
                ok = False
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        self._all_reduce_host(flag, dist.ReduceOp.MIN)
        if int(flag.item()) != 1:
            return False
        self.sum_ch, self.key_ch = chans["sum"], chans["key"]
        self.gather_ch = chans.get("gather")
        return True

    def _close_ipc(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        if dist.is_initialized():
            dist.barrier(group=self.group)
        for p in self._peers:
            p.close()
        if dist.is_initialized():
            dist.barrier(group=self.group)
        for ib in self._inboxes:
            ib.close()
        self._peers, self._inboxes = [], []

    def _selftest(self) -> bool:
        """Two sums and a key max against known answers, bounded by a short timeout."""
        saved, self.timeout_s = self.timeout_s, min(self.timeout_s, 10.0)
        try:
            x = torch.full((self.n,), float(self.rank + 1), device=self.device)
            out = torch.zeros_like(x)
            self.sum_(x, out, accumulate=False)
            self.sum_(x, out, accumulate=True)
            key = torch.tensor([(self.rank + 1) * 7], dtype=torch.int64, device=self.device)
            self.max_key_(key)
            torch.cuda.synchronize(self.device)
            want = self.world * (self.world + 1)
            ok = bool(torch.all(out == float(want))) and int(key.item()) == self.world * 7
            return ok and self.errors() == 0
        finally:
            self.timeout_s = saved

    # -- the decode-step collectives
    def sum_(self, partial: torch.Tensor, out: torch.Tensor, accumulate: bool) -> None:
        """out (+)= sum over ranks of partial (f32 vectors of n)."""
        if self.world == 1:
            if accumulate:
                out.add_(partial)
            elif out.data_ptr() != partial.data_ptr():
                out.copy_(partial)
            return
        if self.mode == "ipc":
            from ..ops import hip as K
            ch = self.sum_ch
            K.ar_sum(partial, out, accumulate, ch["peers"], ch["inbox"].ptr, ch["seq"],
                     ch["err"], self.rank, self.world, self.timeout_s)
            return
        buf = partial.clone()
        self.dense_sum_(buf)
        if accumulate:
            out.add_(buf)
        else:
            out.copy_(buf)

    def max_key_(self, slot: torch.Tensor) -> None:
        """slot (u64 argmax key in an int64 tensor) <- max over ranks."""
        if self.world == 1:
            return
        if self.mode == "ipc":
            from ..ops import hip as K
            ch = self.key_ch
            K.ar_max_key(slot, ch["peers"], ch["inbox"].ptr, ch["seq"], ch["err"], self.rank,
                         self.world, self.timeout_s)
            return
        # signed max of (key XOR sign bit) == unsigned max of key
        flip = torch.tensor(-(1 << 63), dtype=torch.int64, device=slot.device)
        t = torch.bitwise_xor(slot, flip)
        if self.staged and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MAX, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        slot.copy_(torch.bitwise_xor(t, flip))

    def gather_(self, shard: torch.Tensor, off: int, full: torch.Tensor) -> None:
        """full <- the ranks' contiguous shards (this rank's at [off, off + len))."""
        if self.world == 1:
            full.copy_(shard)
            return
        if self.mode == "ipc":
            if self.gather_ch is None:
                raise RuntimeError("AllReduce built without a gather channel (n_gather)")
            from ..ops import hip as K
            ch = self.gather_ch
            K.ar_gather(shard, off, full, ch["peers"], ch["inbox"].ptr, ch["seq"], ch["err"],
                        self.rank, self.world, self.timeout_s)
            return
        full.zero_()
        full[off:off + shard.numel()].copy_(shard)
        self.dense_sum_(full)

    def errors(self) -> int:
        if self.mode != "ipc":
            return 0
        e = int(self.sum_ch["err"].item()) | int(self.key_ch["err"].item())
        if self.gather_ch is not None:
            e |= int(self.gather_ch["err"].item())
        return e

    def measure_us(self, iters: int = 200) -> float | None:
        """Device time of one hidden-size all-reduce (graph of `iters` back to back)."""
        if self.world == 1 or self.device.type != "cuda":
            return None
        x = torch.ones(self.n, device=self.device)
        out = torch.zeros_like(x)
        if self.mode == "ipc":
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(iters):
                    self.sum_(x, out, accumulate=False)
            self.barrier()
            g.replay()
            torch.cuda.synchronize(self.device)
            self.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) * 1e3 / iters
        import time
        self.barrier()
        t0 = time.perf_counter()
        for _ in range(20):
            self.sum_(x, out, accumulate=False)
        torch.cuda.synchronize(self.device)
        return (time.perf_counter() - t0) * 1e6 / 20

    def barrier(self) -> None:
        if dist.is_initialized() and self.world > 1:
            dist.barrier(group=self.group)

    def close(self) -> None:
        if self._inboxes:
            self._close_ipc()


# ---------------------------------------------------------------------------
# engine
# ---------------------------------------------------------------------------
class TPBuffers:
    """Device state of one rank's decode step (graph-stable addresses)."""

    def __init__(self, H, nq, nkv_l, hd, I_l, V_l, max_seq, device, dtype):
        f32, i32 = torch.float32, torch.int32
        self.resid = torch.zeros(H, device=device, dtype=f32)
        self.partial = torch.zeros(H, device=device, dtype=f32)
        self.q = torch.zeros(nq * hd, device=device, dtype=f32)
        self.attn_out = torch.zeros(nq * hd, device=device, dtype=dtype)
        self.act = torch.zeros(I_l, device=device, dtype=dtype)
        self.part = torch.zeros(2 * nq * 64 * (hd + 2), device=device, dtype=f32)
        self.tickets = torch.zeros(2 * nkv_l + 2, device=device, dtype=i32)  # + error word
        self.pos = torch.zeros(1, device=device, dtype=i32)
        self.logits = torch.zeros(V_l, device=device, dtype=f32)
        self.tok = torch.zeros(1, device=device, dtype=i32)
        self.hist = torch.zeros(max_seq, device=device, dtype=i32)
        self.hist_len = torch.zeros(1, device=device, dtype=i32)
        self.slot = torch.zeros(1, device=device, dtype=torch.int64)
        self.thr = torch.zeros(1, device=device, dtype=i32)   # top-k/top-p threshold key


class TPEngine:
    """One rank of a tensor-parallel decoder.  Every rank calls the same methods
    with the same arguments (SPMD); every rank ends with the same tokens."""

    def __init__(self, cfg: LlamaConfig, blocks: dict, head: TPHead, rank: int, world: int,
                 device, dtype, max_seq: int, comm: AllReduce, repeat_penalty: float = 1.0,
                 repeat_last_n: int = 128, temperature: float = 0.0, seed: int = 299792458,
                 use_graph: bool = True):
        check_tp(cfg, world)
        self.cfg, self.rank, self.world = cfg, rank, world
        self.device, self.dtype, self.max_seq = torch.device(device), dtype, max_seq
        self.blocks = dict(sorted(blocks.items()))
        self.head, self.comm = head, comm
        self.penalty, self.last_n = float(repeat_penalty), int(repeat_last_n)
        self.sampling = None         # SamplingConfig of the sampled mode (None = greedy)
        self.params = None           # device SampleParams (hip)
        self.full_logits = None      # gathered vocabulary (sampled mode)
        self._host_sampler = None    # torch path: seeded LogitsProcessor over full logits
        self.hip = self.device.type == "cuda" and dtype in (torch.float16, torch.bfloat16)
        # the torch.distributed fallback issues host collectives: eager launches only
        self.use_graph = use_graph and self.hip and (world == 1 or comm.mode == "ipc")
        H, hd = cfg.hidden_size, cfg.head_dim
        self.nq = cfg.num_attention_heads // world
        self.nkv = cfg.num_key_value_heads // world
        self.I_l = next(iter(self.blocks.values())).wg.shape[0]
        self.V_l = head.lm.shape[0]
        L = len(self.blocks)
        self.kc = torch.zeros((L, self.nkv, max_seq, hd), device=self.device, dtype=dtype)
        self.vc = torch.zeros_like(self.kc)
        self.inv_freq = R.inv_freq(hd, cfg.rope_theta, cfg.rope_scaling).to(self.device)
        self.scale = 1.0 / math.sqrt(hd)
        self.b = TPBuffers(H, self.nq, self.nkv, hd, self.I_l, self.V_l, max_seq, self.device,
                           dtype)
        self.graphs: dict = {}       # mode ("greedy" / "sample") -> {split cap: graph}
        self._graph_sets: dict = {}  # mode -> native-loop GraphSet of those graphs
        self.host_pos = 0
        self.tokens: list[int] = []
        if temperature and temperature > 0:
            from ..models.sampling import SamplingConfig
            self.set_sampling(SamplingConfig(temperature=float(temperature), seed=int(seed),
                                             repeat_penalty=self.penalty,
                                             repeat_last_n=self.last_n))

    # ------------------------------------------------------------------ sampling
    @property
    def mode(self) -> str:
        return "greedy" if self.sampling is None else "sample"

    def set_sampling(self, sampling) -> None:
        """Sampling configuration of the next generation (every rank, same value; None or
        temperature <= 0 = greedy).  hip: rewrites the device parameter block only —
        the captured graphs of the mode are replayed as they are."""
        from ..models.sampling import LogitsProcessor
        self.sampling = sampling if sampling is not None and not sampling.greedy else None
        if self.sampling is None:
            self._host_sampler = None
            return
        if self.hip:
            from ..ops import hip as K
            if self.params is None:
                self.params = torch.zeros(K.SAMPLE_PARAMS_WORDS, dtype=torch.int32,
                                          device=self.device)
            self.params.copy_(K.pack_sample_params(self.sampling))
        else:
            self._host_sampler = LogitsProcessor(self.sampling)
        if self.full_logits is None:
            self.full_logits = torch.zeros(self.cfg.vocab_size, device=self.device,
                                           dtype=torch.float32)

    # ------------------------------------------------------------------ prefill
    def prefill(self, prompt: list[int]) -> int:
        """Fill this rank's KV heads for the prompt; returns the first token."""
        cfg, T = self.cfg, len(prompt)
        if T + 1 > self.max_seq:
            raise ValueError("prompt longer than max_seq")
        ids = torch.tensor(prompt, dtype=torch.long, device=self.device)
        h = self.head.embed[ids].float()
        for s, (li, w) in enumerate(self.blocks.items()):
            if self.hip:
                self._prefill_block_hip(h, w, s)
            else:
                self._prefill_block_torch(h, w, s)
        self.tokens = list(prompt)
        b = self.b
        if self.hip:
            b.hist[:T].copy_(ids.int())
            b.hist_len.fill_(T)
            b.pos.fill_(T - 1)
            b.slot.zero_()
            self._head_hip(h[-1].contiguous())
            tok = int(b.tok.item())
        else:
            tok = self._head_torch(h[-1])
            b.pos.fill_(T)
        self.host_pos = T
        self.tokens.append(tok)
        return tok

    def _prefill_block_hip(self, h, w, s):
        from ..ops import gemm as G
        from ..ops import hip as K
        cfg, T = self.cfg, h.shape[0]
        hd, nq, nkv = cfg.head_dim, self.nq, self.nkv
        x = torch.empty((T, cfg.hidden_size), device=h.device, dtype=self.dtype)
        K.rmsnorm(h, w.ln1, cfg.rms_norm_eps, x)
        qkv = G.linear(x, w.wqkv)
        q, k, v = qkv[:, :nq * hd], qkv[:, nq * hd:(nq + nkv) * hd], qkv[:, (nq + nkv) * hd:]
        K.rope_kv(q, k, v, self.inv_freq, 0, self.kc[s], self.vc[s])
        att = torch.empty((T, nq * hd), device=h.device, dtype=self.dtype)
        K.flash_attn(q.view(1, T, nq, hd).transpose(1, 2), self.kc[s][None, :, :T],
                     self.vc[s][None, :, :T], att.view(1, T, nq, hd).transpose(1, 2), self.scale,
                     causal=True, pos0=0)
        part = torch.empty_like(h)
        G.linear(att, w.wo, epi="store32", resid=part)
        self.comm.dense_sum_(part)
        h += part
        K.rmsnorm(h, w.ln2, cfg.rms_norm_eps, x)
        act = G.linear(x, w.wgu, epi="swiglu")
        G.linear(act, w.wd, epi="store32", resid=part)
        self.comm.dense_sum_(part)
        h += part

    def _prefill_block_torch(self, h, w, s):
        cfg, T, dt = self.cfg, h.shape[0], self.dtype
        hd, nq, nkv = cfg.head_dim, self.nq, self.nkv
        pos = torch.arange(T, device=h.device)
        x = R.rms_norm(h, w.ln1, cfg.rms_norm_eps).to(dt)
        q = R.rope((x @ w.wq.t()).view(T, nq, hd), pos, self.inv_freq).to(dt)
        k = R.rope((x @ w.wk.t()).view(T, nkv, hd), pos, self.inv_freq).to(dt)
        v = (x @ w.wv.t()).view(T, nkv, hd).to(dt)
        self.kc[s, :, :T] = k.transpose(0, 1)
        self.vc[s, :, :T] = v.transpose(0, 1)
        att = R.attention(q, k, v, 0).to(dt).reshape(T, nq * hd)
        part = (att @ w.wo.t()).float()
        self.comm.dense_sum_(part)
        h += part
        x2 = R.rms_norm(h, w.ln2, cfg.rms_norm_eps).to(dt)
        act = R.silu_mul(x2 @ w.wg.t(), x2 @ w.wu.t()).to(dt)
        part = (act @ w.wd.t()).float()
        self.comm.dense_sum_(part)
        h += part

    # ------------------------------------------------------------------ head
    def _head_hip(self, row: torch.Tensor) -> None:
        """ln_f + this rank's lm_head rows, then the token: greedy = shard argmax key ->
        global max; sampled = gather the full vocabulary -> the single-GPU device
        selection with the parameter block (identical on every rank)."""
        from ..ops import hip as K
        b = self.b
        K.norm_gemv_f32(row, self.head.norm, self.cfg.rms_norm_eps, self.head.lm, b.logits)
        if self.sampling is None:
            K.select_shard(b.logits, self.head.voff, b.hist, b.hist_len, self.last_n,
                           self.penalty, 0.0, 0, b.slot)
            self.comm.max_key_(b.slot)
            K.finalize_token(b.slot, b.tok, b.hist, b.hist_len, b.pos)
            return
        full = self.full_logits
        self.comm.gather_(b.logits, self.head.voff, full)
        if self.penalty != 1.0:
            K.repeat_penalty(full, b.hist, b.hist_len, self.last_n, self.penalty)
        K.select_token(full, b.slot, b.hist, b.hist_len, b.tok, b.pos, thr=b.thr,
                       params=self.params)

    def _head_torch(self, row: torch.Tensor) -> int:
        x = R.rms_norm(row, self.head.norm, self.cfg.rms_norm_eps).to(self.dtype)
        logits = (x @ self.head.lm.t()).float()
        if self.sampling is not None:   # every rank: same full logits, same seeded draw
            full = self.full_logits
            self.comm.gather_(logits, self.head.voff, full)
            if self.penalty != 1.0:
                full = R.apply_repeat_penalty(full.clone(), self.penalty,
                                              self.tokens[-self.last_n:])
            return int(self._host_sampler.sample(full))
        if self.penalty != 1.0:
            recent = [t - self.head.voff for t in self.tokens[-self.last_n:]]
            recent = [t for t in dict.fromkeys(recent) if 0 <= t < logits.numel()]
            if recent:
                idx = torch.tensor(recent, dtype=torch.long)
                s = logits[idx]
                logits[idx] = torch.where(s >= 0, s / self.penalty, s * self.penalty)
        i = int(torch.argmax(logits))
        v = float(logits[i])
        u = torch.tensor([v], dtype=torch.float32).view(torch.int32).item() & 0xFFFFFFFF
        ordered = (~u & 0xFFFFFFFF) if u & 0x80000000 else (u | 0x80000000)
        key = (ordered << 32) | (0xFFFFFFFF - (i + self.head.voff))
        if key >= 1 << 63:
            key -= 1 << 64
        slot = torch.tensor([key], dtype=torch.int64)
        self.comm.max_key_(slot)
        k = int(slot.item()) & 0xFFFFFFFFFFFFFFFF
        return 0xFFFFFFFF - (k & 0xFFFFFFFF)

    # ------------------------------------------------------------------ decode
    def _step_body(self) -> None:
        from ..ops import hip as K
        cfg, b, comm = self.cfg, self.b, self.comm
        eps = cfg.rms_norm_eps
        K.embed(self.head.embed, b.tok, b.resid)
        for s, w in enumerate(self.blocks.values()):
            K.qkv_rope(b.resid, w.ln1, eps, w.wq, w.wk, w.wv, self.inv_freq, b.pos, b.q,
                       self.kc[s], self.vc[s])
            K.attn_decode(b.q, self.kc[s], self.vc[s], b.pos, self.scale, b.part, b.tickets,
                          b.attn_out)
            if comm.world == 1:  # nothing to reduce: accumulate in place (no sum launch)
                K.gemv(b.attn_out, w.wo, b.resid, accumulate=True)
                K.swiglu(b.resid, w.ln2, eps, w.wg, w.wu, b.act)
                K.gemv(b.act, w.wd, b.resid, accumulate=True)
                continue
            K.gemv(b.attn_out, w.wo, b.partial, accumulate=False)
            comm.sum_(b.partial, b.resid, accumulate=True)
            K.swiglu(b.resid, w.ln2, eps, w.wg, w.wu, b.act)
            K.gemv(b.act, w.wd, b.partial, accumulate=False)
            comm.sum_(b.partial, b.resid, accumulate=True)
        self._head_hip(b.resid)

    def capture(self) -> None:
        """Capture the decode step of the current mode (greedy / sampled) as graphs,
        one per attention split cap (after prefill; every rank together, in the same
        mode).  The warm-up step's token state is restored afterwards; the K/V row it
        wrote is the one the first real step rewrites with the same values."""
        if not self.use_graph or self.mode in self.graphs:
            return
        b = self.b
        saved = [t.clone() for t in (b.tok, b.pos, b.hist_len, b.hist, b.slot)]
        self._step_body()  # warm-up (all ranks: the collectives pair up)
        torch.cuda.synchronize(self.device)
        for t, v in zip((b.tok, b.pos, b.hist_len, b.hist, b.slot), saved):
            t.copy_(v)
        # one graph per attention split cap (position buckets, as DeviceDecoder.capture);
        # every rank picks the same one from the same host position
        from ..ops import hip as K
        gs = {}
        for cap in K.attn_split_caps(self.max_seq):
            g = torch.cuda.CUDAGraph()
            with K.attn_split_cap(cap), torch.cuda.graph(g):
                self._step_body()
            gs[cap] = g
        self.graphs[self.mode] = gs
        torch.cuda.synchronize(self.device)

    def graph_set(self):
        """The current mode's bucket graphs as a native-loop GraphSet."""
        gs = self.graphs[self.mode]
        cur = self._graph_sets.get(self.mode)
        if cur is None or cur.graphs[-1] is not gs[max(gs)]:
            from ..ops import graph_loop as GL
            caps = sorted(gs)
            idx = {id(gs[c]): i for i, c in enumerate(caps)}
            cur = self._graph_sets[self.mode] = GL.GraphSet(
                [gs[c] for c in caps], lambda t: idx[id(self._graph_for(t))], self.max_seq)
        return cur

    def _graph_for(self, tk: int):
        from ..ops import hip as K
        gs = self.graphs[self.mode]
        need = K.attn_splits(tk)
        return next((gs[c] for c in sorted(gs) if c >= need), gs[max(gs)])

    def launch(self) -> None:
        """Enqueue one decode step (async on the HIP path).  Raises instead of writing
        past the KV cache / token history (max_seq)."""
        if self.host_pos + 1 >= self.max_seq:
            raise ValueError(f"decode step at position {self.host_pos} overruns max_seq "
                             f"{self.max_seq}")
        if self.hip:
            if self.use_graph and self.mode in self.graphs:
                self._graph_for(self.host_pos + 2).replay()
            else:
                self._step_body()
        else:
            self._step_torch()
        self.host_pos += 1

    def token(self) -> int:
        if self.hip:
            return int(self.b.tok.item())
        return self.tokens[-1]

    def step(self) -> int:
        self.launch()
        t = self.token()
        if self.hip:
            self.tokens.append(t)
        return t

    def _step_torch(self) -> None:
        cfg, dt = self.cfg, self.dtype
        hd, nq, nkv = cfg.head_dim, self.nq, self.nkv
        pos = self.host_pos
        tok = self.tokens[-1]
        h = self.head.embed[tok].float().view(1, -1)
        p = torch.tensor([pos], device=h.device)
        for s, w in enumerate(self.blocks.values()):
            x = R.rms_norm(h, w.ln1, cfg.rms_norm_eps).to(dt)
            q = R.rope((x @ w.wq.t()).view(1, nq, hd), p, self.inv_freq).to(dt)
            k = R.rope((x @ w.wk.t()).view(1, nkv, hd), p, self.inv_freq).to(dt)
            v = (x @ w.wv.t()).view(1, nkv, hd).to(dt)
            self.kc[s, :, pos] = k[0]
            self.vc[s, :, pos] = v[0]
            att = R.attention(q, self.kc[s, :, :pos + 1].transpose(0, 1),
                              self.vc[s, :, :pos + 1].transpose(0, 1), pos).to(dt)
            part = (att.reshape(1, nq * hd) @ w.wo.t()).float()
            self.comm.dense_sum_(part)
            h += part
            x2 = R.rms_norm(h, w.ln2, cfg.rms_norm_eps).to(dt)
            act = R.silu_mul(x2 @ w.wg.t(), x2 @ w.wu.t()).to(dt)
            part = (act @ w.wd.t()).float()
            self.comm.dense_sum_(part)
            h += part
        self.tokens.append(self._head_torch(h[0]))

    def decode(self, n: int) -> list[int]:
        """n more tokens (after prefill)."""
        return [self.step() for _ in range(n)]

    def check(self) -> None:
        if self.comm.errors():
            raise RuntimeError("tensor-parallel all-reduce timed out (a peer stopped?)")
        if self.hip:
            from ..ops import hip as K
            if K.attn_error(self.b.tickets):
                K.attn_clear_error(self.b.tickets)
                raise RuntimeError(f"tensor-parallel rank {self.rank}: decode attention split "
                                   "merge timed out; outputs of that launch are invalid")

    def close(self) -> None:
        self.comm.close()
