"""Layer-sharded decode pipeline over RCCL point-to-point (one process per GPU).

This is the MI355X data plane for cake's master → worker → master hop
(cake-core/src/models/llama3/llama.rs:95-114 and client.rs:116-124, which send a
``Batch{x, [(layer, index_pos, block_idx)]}`` frame over TCP and copy the
tensor device→host→device on both ends, proto/message.rs:22-38).  Here:

* The placement is a list of *runs* (consecutive layers with one owner rank,
  i.e. contiguous-block batching); rank 0 is the master (embedding, ln_f,
  lm_head, sampling) and may own runs too.
* A hop is ONE device-to-device RCCL send/recv of a message
  ``[hidden (H f32) | header (16 x int32)]`` — header word 0 is the position,
  word 1 the stream (sequence) id — so the receiving rank's hipGraph reads
  the position straight out of the received buffer: no host round trip, no
  descriptor message for decode.  Prefill (T>1) sends an int32 header, then
  the [T, H] block.
* ``streams`` independent sequences can be in flight: while rank r runs
  stream s, rank r-1 already runs stream s+1 (the reference's global API lock
  allows one).  With streams = 1 it is exactly cake's sequential pipeline.
* Backends: ``hip`` (graph per stream per run, RCCL via torch.distributed
  backend "nccl") or ``torch`` (eager reference math; gloo on CPU for tests).
* Decode hops (``hop``): ``"dist"`` — host-issued torch.distributed p2p
  between graph replays (RCCL over xGMI, or host-staged gloo); ``"ipc"`` —
  device-side peer stores into the next rank's inbox (parallel/hop.py,
  csrc/kernels/hop.hip), captured INSIDE each rank's decode graph, so a rank's
  whole token (receive -> its layers -> send) is one replay and no host is on
  the critical path.  Prefill always uses the dist path.
* Every decode graph is captured once per attention split cap (position
  buckets, as the single-GPU DeviceDecoder): all ranks track the live length
  on the host (``_Stream.dev_pos``) and replay the smallest cap covering it.
* Serving (:meth:`PipelineEngine.serve` / :meth:`PipelineEngine.generate`): the
  master gates every unit of work with a host control message on a separate
  gloo group (``prefill``, ``decode n``, ``stop``) — an idle worker blocks on
  the host, never inside a device-side receive — and workers enqueue ``n``
  token replays per ``decode`` message, so with ipc hops a chunk of tokens runs
  with no host in the loop; the master reads tokens back one replay behind.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass

import torch
import torch.distributed as dist

from ..models.llama3.blocks import DecodeBuffers, LayerStack
from ..models.llama3.config import LlamaConfig
from ..models.llama3.weights import HeadWeights
from ..ops import reference as R


def init_process_group(backend: str, rank: int, world: int, device=None) -> None:
    """torch.distributed init with a bounded collective timeout (CAKE_DIST_TIMEOUT s,
    default 600) and asynchronous error handling, so a dead peer surfaces as an
    error on the other ranks instead of a hang."""
    import datetime
    import os
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    timeout = datetime.timedelta(seconds=float(os.environ.get("CAKE_DIST_TIMEOUT", "600")))
    kw = {"device_id": device} if backend == "nccl" and device is not None else {}
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=timeout, **kw)


HDR = 16          # int32 header words appended to each hop message
H_POS, H_STREAM, H_T, H_FLAGS = 0, 1, 2, 3
FLAG_RESET, FLAG_PREFILL, FLAG_STOP = 1, 2, 4


def shard_layers(num_layers: int, world: int, head_cost: float = 0.0) -> list[list[int]]:
    """Contiguous shards (rank r gets layers [a_r, b_r)) balancing per-rank work.

    ``head_cost`` is the master's extra work (embedding + ln_f + lm_head +
    sampling) in units of one transformer block; rank 0 then gets that many
    fewer blocks.  With head_cost = 0 this is a near-equal split.
    """
    if world == 1:
        return [list(range(num_layers))]
    total = num_layers + head_cost
    out, start = [], 0
    for r in range(world):
        # cumulative target boundary after rank r (in block units incl. the head)
        end = round((r + 1) * total / world - head_cost) if r < world - 1 else num_layers
        end = max(start + (1 if num_layers - start >= world - r else 0), min(end, num_layers - (world - 1 - r)))
        out.append(list(range(start, end)))
        start = end
    return out


def head_cost_in_layers(cfg) -> float:
    """lm_head bytes relative to one block's weight bytes (decode is bandwidth-bound)."""
    return (cfg.vocab_size * cfg.hidden_size * 2) / cfg.layer_bytes(2)


@dataclass
class PipeRun:
    owner: int
    layers: list[int]


def plan_from_owners(owners: list[int]) -> list[PipeRun]:
    """owners[l] = rank executing layer l -> runs of consecutive equal owners."""
    runs: list[PipeRun] = []
    for li, r in enumerate(owners):
        if runs and runs[-1].owner == r:
            runs[-1].layers.append(li)
        else:
            runs.append(PipeRun(r, [li]))
    return runs


class _Stream:
    """Per-sequence device state on one rank."""

    def __init__(self, eng: "PipelineEngine", sid: int):
        H = eng.cfg.hidden_size
        self.sid = sid
        self.msg = torch.zeros(H + HDR, device=eng.device, dtype=torch.float32)
        self.resid = self.msg[:H]
        self.hdr = self.msg[H:].view(torch.int32)
        self.bufs = DecodeBuffers(eng.cfg, eng.stack.max_seq, eng.device, eng.stack.dtype,
                                  with_head=eng.is_master, resid=self.resid,
                                  pos=self.hdr[H_POS:H_POS + 1])
        self.graphs: dict = {}     # body key -> {split cap: graph}
        self.send_work = None
        self.host_tokens: list[int] = []   # torch backend bookkeeping (master)
        self.host_pos = 0
        self.dev_pos = 0   # position of the next decode token (host mirror, every rank)


class PipelineEngine:
    def __init__(self, cfg: LlamaConfig, stack: LayerStack, owners: list[int], rank: int,
                 world: int, streams: int = 1, head: HeadWeights | None = None,
                 repeat_penalty: float = 1.0, repeat_last_n: int = 128, use_graph: bool = True,
                 group=None, hop: str = "dist", hop_bf16: bool = False,
                 steps_per_graph: int = 1):
        self.cfg, self.stack, self.rank, self.world = cfg, stack, rank, world
        self.device = stack.device
        self.is_master = rank == 0
        self.head = head
        if self.is_master and head is None:
            raise ValueError("rank 0 (master) needs the head weights")
        self.runs = plan_from_owners(owners)
        self.my_runs = [j for j, r in enumerate(self.runs) if r.owner == rank]
        for j in self.my_runs:
            missing = [li for li in self.runs[j].layers if li not in stack.weights]
            if missing:
                raise ValueError(f"rank {rank} lacks weights for layers {missing}")
        self.penalty, self.last_n = float(repeat_penalty), int(repeat_last_n)
        self.sampler = None   # host sampler (torch backend); None = selection on the device
        self.sampling = None  # SamplingConfig for the device draw (temperature > 0)
        self.sample_params = None  # device SampleParams (set_sampling): per-request config
        self.hip = stack.backend == "hip"
        self.use_graph = use_graph and self.hip
        self.group = group
        # gloo with device tensors (1-GPU multi-process tests): stage via the host
        self.staged = dist.is_initialized() and dist.get_backend(group) == "gloo"
        # Hops toward a higher rank and toward a lower rank use two different
        # communicators (own RCCL comm + stream each), so two ranks exchanging in
        # both directions never serialise a send behind a recv on one stream —
        # the schedule is deadlock-free even with rendezvous (unbuffered) sends.
        self.g_up = self.g_down = group
        if dist.is_initialized() and world > 1:
            ranks = list(range(world))
            self.g_up = dist.new_group(ranks)
            self.g_down = dist.new_group(ranks)
        if stack.max_sessions < streams:
            stack.max_sessions = streams
        self.streams = [_Stream(self, s) for s in range(streams)]
        if hop not in ("dist", "ipc"):
            raise ValueError(f"unknown hop transport {hop}")
        self.hop = "dist"
        self.hop_bf16 = bool(hop_bf16)
        self.k = max(1, int(steps_per_graph))
        self._skip_hops = False
        self._events: list = []
        self.inbox, self.peer = {}, {}
        # host control plane of serve()/generate(): its own gloo group, whose timeout
        # bounds how long a worker may sit idle between requests
        self.ctrl = None
        if dist.is_initialized() and world > 1:
            import datetime
            idle = float(os.environ.get("CAKE_SERVE_IDLE_TIMEOUT", str(7 * 86400)))
            self.ctrl = dist.new_group(list(range(world)), backend="gloo",
                                       timeout=datetime.timedelta(seconds=idle))
        if hop == "ipc" and world > 1 and self.use_graph and dist.is_initialized():
            self._setup_ipc()  # (ipc hops need the hip backend with graphs: else dist)

    # ------------------------------------------------------------------ hop helpers
    def _prev(self, j: int) -> int:
        return self.runs[j - 1].owner if j > 0 else 0

    def _next(self, j: int) -> int:
        return self.runs[j + 1].owner if j + 1 < len(self.runs) else 0

    def _first_dst(self) -> int:
        """Rank the master sends a freshly embedded token to."""
        return self.runs[0].owner if self.runs[0].owner != 0 else self._next(0)

    def _final_src(self) -> int:
        """Rank the master receives the finished hidden state from."""
        last = len(self.runs) - 1
        if self.runs[last].owner != 0:
            return self.runs[last].owner
        return self.runs[last - 1].owner if last > 0 else 0

    # ------------------------------------------------------------------ ipc hops
    # Stage k of a token: 0 = head (master: embed), 1..R = run k-1, R+1 = tail
    # (master: ln_f, lm_head, token selection).  A hop precedes stage k when its
    # owner differs from stage k-1's.
    def _stage_owner(self, k: int) -> int:
        R = len(self.runs)
        return 0 if k == 0 or k == R + 1 else self.runs[k - 1].owner

    def _recv_point(self, k: int) -> bool:
        return k > 0 and self._stage_owner(k) != self._stage_owner(k - 1)

    def _setup_ipc(self) -> None:
        """Allocate this rank's inboxes, exchange IPC handles, map the peers' inboxes,
        then prove every link with one tagged message (fall back to dist hops on
        any failure, agreed by all ranks)."""
        from . import hop as HP
        H = self.cfg.hidden_size
        R = len(self.runs)
        self._H = H
        words = HP.hop_words(H, HDR, self.hop_bf16)
        n_st = len(self.streams)
        ok = 1
        self.inbox, self.peer = {}, {}
        try:
            mine = {}
            for st in self.streams:
                for k in range(1, R + 2):
                    if self._recv_point(k) and self._stage_owner(k) == self.rank:
                        ib = HP.Inbox(words)
                        self.inbox[(st.sid, k)] = ib
                        mine[(st.sid, k)] = ib.handle()
        except Exception as e:  # noqa: BLE001  (reported, then agreed on below)
            print(f"[pipeline] rank {self.rank}: inbox setup failed: {e}", file=sys.stderr, flush=True)
            ok, mine = 0, {}
        allh = [None] * self.world
        dist.all_gather_object(allh, mine)
        try:
            if ok:
                for st in self.streams:
                    for k in range(1, R + 2):
                        if self._recv_point(k) and self._stage_owner(k - 1) == self.rank:
                            owner = self._stage_owner(k)
                            self.peer[(st.sid, k)] = HP.PeerInbox(allh[owner][(st.sid, k)])
        except Exception as e:  # noqa: BLE001
            print(f"[pipeline] rank {self.rank}: ipc open failed: {e}", file=sys.stderr, flush=True)
            ok = 0
        # per (stream, stage) sequence counters (sender side and receiver side) + error word
        self._seq = torch.zeros(2 * n_st * (R + 2), dtype=torch.int32, device=self.device)
        self._err = torch.zeros(1, dtype=torch.int32, device=self.device)
        if ok:
            ok = int(self._ipc_selftest())
        flag = torch.tensor([ok], dtype=torch.int32,
                            device=self.device if dist.get_backend(self.group) == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 1:
            self.hop = "ipc"
            return
        if self.rank == 0:
            print("[pipeline] ipc hops unavailable on some rank: using dist hops", file=sys.stderr, flush=True)
        for t in list(self.peer.values()) + list(self.inbox.values()):
            t.close()
        self.inbox, self.peer = {}, {}

    def _seq_t(self, sid: int, k: int, side: int) -> torch.Tensor:
        R = len(self.runs)
        i = (side * len(self.streams) + sid) * (R + 2) + k
        return self._seq[i:i + 1]

    def _ipc_send(self, st: "_Stream", k: int) -> None:
        from . import hop as HP
        HP.send(st.msg, self._H, HDR, self.hop_bf16, self.peer[(st.sid, k)],
                self._seq_t(st.sid, k, 0))

    def _ipc_recv(self, st: "_Stream", k: int, timeout_s: float | None = None) -> None:
        from . import hop as HP
        HP.recv(self.inbox[(st.sid, k)], st.msg, self._H, HDR, self.hop_bf16,
                self._seq_t(st.sid, k, 1), self._err, timeout_s)

    def _ipc_selftest(self) -> bool:
        """One tagged message over every link (a known pattern, short timeout);
        the message buffers and sequence counters are restored afterwards."""
        R = len(self.runs)
        saved = [st.msg.clone() for st in self.streams]
        try:
            for st in self.streams:
                pat = torch.arange(st.msg.numel(), device=self.device, dtype=torch.float32)
                pat = pat * 0.25 + 1000 * self.rank + st.sid
                for k in range(1, R + 2):
                    if not self._recv_point(k):
                        continue
                    src, dst = self._stage_owner(k - 1), self._stage_owner(k)
                    if src == dst:
                        continue
                    if src == self.rank:
                        st.msg.copy_(pat)
                        self._ipc_send(st, k)
                    if dst == self.rank:
                        self._ipc_recv(st, k, timeout_s=20.0)
                        torch.cuda.synchronize(self.device)
                        exp = (torch.arange(st.msg.numel(), device=self.device,
                                            dtype=torch.float32) * 0.25 + 1000 * src + st.sid)
                        H = self._H
                        got_h, exp_h = st.msg[:H], exp[:H]
                        if self.hop_bf16:
                            exp_h = exp_h.to(torch.bfloat16).float()
                        if int(self._err.item()) != 0 or not torch.equal(got_h, exp_h) or \
                                not torch.equal(st.msg[H:].view(torch.int32),
                                                exp[H:].view(torch.int32)):
                            print(f"[pipeline] rank {self.rank}: ipc self-test mismatch on "
                                  f"stage {k}", file=sys.stderr, flush=True)
                            return False
                    torch.cuda.synchronize(self.device)
            return True
        except Exception as e:  # noqa: BLE001
            print(f"[pipeline] rank {self.rank}: ipc self-test failed: {e}", file=sys.stderr, flush=True)
            return False
        finally:
            torch.cuda.synchronize(self.device)
            for st, v in zip(self.streams, saved):
                st.msg.copy_(v)
            self._err.zero_()

    def _ipc_stages(self) -> list[int]:
        return [k for k in range(len(self.runs) + 2) if self._stage_owner(k) == self.rank]

    def _ipc_stage_body(self, st: "_Stream", k: int) -> None:
        """Stage k of one token for stream st on this rank (graph-capturable)."""
        from ..ops import hip as K
        R = len(self.runs)
        if self._recv_point(k) and not self._skip_hops:
            self._ipc_recv(st, k)
        if k == 0:
            K.embed(self.head.embed, st.bufs.tok, st.resid)
        elif k == R + 1:
            b = st.bufs
            if (self.sampler is None and self.sampling is None and self.sample_params is None
                    and (self.penalty == 1.0 or self.last_n <= K.HEAD_SELECT_MAX_LAST_N)
                    and os.environ.get("CAKE_FUSED_HEAD", "1") != "0"):
                # greedy: lm_head + penalty + argmax + finalize in one launch
                K.head_select(st.resid, self.head.norm, self.cfg.rms_norm_eps,
                              self.head.lm_head, b.logits, b.hist, b.hist_len,
                              self.last_n if self.penalty != 1.0 else 0, self.penalty,
                              b.slot, b.sel_ticket, b.tok, b.pos)
            else:
                K.norm_gemv_f32(st.resid, self.head.norm, self.cfg.rms_norm_eps,
                                self.head.lm_head, b.logits)
                self._select_device(st)
        else:
            self.stack.decode_step(st.bufs, self.runs[k - 1].layers, st.sid)
        if k < R + 1 and self._recv_point(k + 1) and not self._skip_hops:
            self._ipc_send(st, k + 1)

    def _ipc_token_body(self, st: "_Stream") -> None:
        for k in self._ipc_stages():
            self._ipc_stage_body(st, k)

    def hops_per_token(self) -> int:
        return sum(1 for k in range(1, len(self.runs) + 2) if self._recv_point(k))

    def close(self) -> None:
        """Collective: unmap the peers' inboxes, free this rank's, drop the extra groups."""
        if self.hip:
            torch.cuda.synchronize(self.device)
        if self.inbox or self.peer:
            dist.barrier(group=self.group)
            for t in self.peer.values():
                t.close()
            dist.barrier(group=self.group)
            for t in self.inbox.values():
                t.close()
            self.inbox, self.peer = {}, {}
        for st in self.streams:
            st.graphs = {}
        for g in (self.g_up, self.g_down, self.ctrl):
            if g is not None and g is not self.group:
                try:
                    dist.destroy_process_group(g)
                except Exception:  # noqa: BLE001  (best effort at teardown)
                    pass
        self.g_up = self.g_down = self.group
        self.ctrl = None

    def check_hops(self) -> None:
        """Raise if any device-side receive timed out (a peer stopped sending)."""
        if self.hop == "ipc" and int(self._err.item()) != 0:
            raise RuntimeError(f"rank {self.rank}: a pipeline hop timed out "
                               f"(CAKE_HOP_TIMEOUT={os.environ.get('CAKE_HOP_TIMEOUT', '60')} s)")
        if self.hip:
            for st in self.streams:
                self.stack.mk_check(st.bufs)

    def measure_hop_us(self, iters: int = 100) -> float | None:
        """One-way latency of a decode hop between ranks 0 and 1 (ping-pong; µs).
        All ranks call it; ranks >= 2 only join the barriers.  None if world == 1."""
        if self.world < 2:
            return None
        H = self.cfg.hidden_size
        msg = torch.zeros(H + HDR, device=self.device, dtype=torch.float32)
        reps = 10
        if self.hop == "ipc":
            from . import hop as HP
            words = HP.hop_words(H, HDR, self.hop_bf16)
            ib = HP.Inbox(words) if self.rank in (0, 1) else None
            allh = [None] * self.world
            dist.all_gather_object(allh, ib.handle() if ib is not None else None)
            peer = HP.PeerInbox(allh[1 - self.rank]) if self.rank in (0, 1) else None
            seq = torch.zeros(2, dtype=torch.int32, device=self.device)
            err = torch.zeros(1, dtype=torch.int32, device=self.device)

            def body():
                for _ in range(iters):
                    if self.rank == 0:
                        HP.send(msg, H, HDR, self.hop_bf16, peer, seq[0:1])
                        HP.recv(ib, msg, H, HDR, self.hop_bf16, seq[1:2], err)
                    else:
                        HP.recv(ib, msg, H, HDR, self.hop_bf16, seq[1:2], err)
                        HP.send(msg, H, HDR, self.hop_bf16, peer, seq[0:1])
            g = None
            if self.rank in (0, 1):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    body()
            dist.barrier(group=self.group)
            torch.cuda.synchronize(self.device)
            t = None
            if g is not None:
                g.replay()  # warm
                torch.cuda.synchronize(self.device)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    g.replay()
                e1.record()
                e1.synchronize()
                t = e0.elapsed_time(e1) * 1e3 / (reps * iters * 2)
                if int(err.item()) != 0:
                    t = None
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.group)
            if peer is not None:
                peer.close()
            dist.barrier(group=self.group)
            if ib is not None:
                ib.close()
            return t
        # host-issued dist p2p ping-pong
        import time
        dist.barrier(group=self.group)
        t0 = time.perf_counter()
        n = iters * 2
        for _ in range(n // 2):
            if self.rank == 0:
                self._wait(self._send(msg, 1))
                self._recv(msg, 1)
            elif self.rank == 1:
                self._recv(msg, 0)
                self._wait(self._send(msg, 0))
        if msg.is_cuda:
            torch.cuda.synchronize(self.device)
        dt = (time.perf_counter() - t0) * 1e6 / n
        dist.barrier(group=self.group)
        return dt if self.rank in (0, 1) else None

    def _send(self, t: torch.Tensor, dst: int):
        g = self.g_up if dst > self.rank else self.g_down
        if self.staged and t.is_cuda:
            host = t.to("cpu")          # gloo moves host memory only: stage through the host
            return dist.isend(host, dst, group=g)
        return dist.isend(t, dst, group=g)

    def _recv(self, t: torch.Tensor, src: int) -> None:
        g = self.g_up if src < self.rank else self.g_down
        if self.staged and t.is_cuda:
            host = torch.empty(t.shape, dtype=t.dtype)
            dist.irecv(host, src, group=g).wait()
            t.copy_(host)
            return
        dist.irecv(t, src, group=g).wait()

    @staticmethod
    def _wait(work) -> None:
        if work is not None:
            work.wait()

    # ------------------------------------------------------------------ master head ops
    def _embed(self, tokens, out: torch.Tensor) -> None:
        if self.hip:
            from ..ops import hip as K
            K.embed(self.head.embed, tokens, out)
        else:
            out.copy_(self.head.embed[tokens.long()].float().view_as(out))

    def _logits(self, row: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if self.hip:
            from ..ops import hip as K
            if out is None:
                out = torch.empty(self.cfg.vocab_size, device=self.device)
            K.norm_gemv_f32(row, self.head.norm, self.cfg.rms_norm_eps, self.head.lm_head, out)
            return out
        x = R.rms_norm(row, self.head.norm, self.cfg.rms_norm_eps).to(self.stack.dtype)
        return (x @ self.head.lm_head.t()).float()

    def _select_host(self, st: _Stream, logits: torch.Tensor) -> int:
        if self.penalty != 1.0:
            logits = R.apply_repeat_penalty(logits, self.penalty, st.host_tokens[-self.last_n:])
        if self.sampler is not None:
            return int(self.sampler(logits))
        return int(torch.argmax(logits))

    def _select_device(self, st: _Stream) -> None:
        """Penalty + token selection (argmax, or the seeded device draw when
        ``self.sampling`` is set) + next-token bookkeeping, on the device."""
        from ..ops import hip as K
        b = st.bufs
        if self.penalty != 1.0:
            K.repeat_penalty(b.logits, b.hist, b.hist_len, self.last_n, self.penalty)
        if self.sampler is None:
            K.select_token(b.logits, b.slot, b.hist, b.hist_len, b.tok, b.pos, self.sampling,
                           b.thr, params=self.sample_params)

    def set_sampling(self, sampling) -> None:
        """Per-request sampling (API temperature / top_k / top_p; None or temperature
        <= 0 = greedy).  hip: the selection reads a device parameter block, so the
        captured graphs stay valid; call once before capture() to switch to it."""
        if not self.is_master:
            return
        if not self.hip:
            from ..models.sampling import LogitsProcessor
            self.sampler = None if sampling is None or sampling.greedy else \
                LogitsProcessor(sampling).sample
            return
        from ..ops import hip as K
        if self.sample_params is None:
            if any(st.graphs for st in self.streams):
                raise RuntimeError("set_sampling: call before capture()")
            self.sample_params = torch.zeros(K.SAMPLE_PARAMS_WORDS, dtype=torch.int32,
                                             device=self.device)
        self.sampler = None
        self.sampling = sampling if sampling is not None and not sampling.greedy else None
        self.sample_params.copy_(K.pack_sample_params(sampling))

    def _host_sample_device(self, st: _Stream) -> int:
        """Sampled decoding on the hip path: draw on the host, push to the device state."""
        from ..ops import hip as K
        tok = int(self.sampler(st.bufs.logits))
        src = torch.tensor([tok], dtype=torch.int32, device=self.device)
        b = st.bufs
        K.push_token(src, b.tok, b.hist, b.hist_len, b.pos)
        return tok

    # ------------------------------------------------------------------ prefill
    def prefill(self, sid: int, prompt: list[int] | None = None) -> int | None:
        """Prefill one stream through the pipeline.  Master passes the prompt and
        gets the first generated token; workers pass nothing."""
        st = self.streams[sid]
        H = self.cfg.hidden_size
        self.stack.reset(sid)
        # control header travels in the stream's hop message (flags = PREFILL|RESET)
        hdr = st.hdr
        if self.is_master:
            T = len(prompt)
            if T == 0 or T + 1 > self.stack.max_seq:
                raise ValueError(f"prompt of {T} tokens does not fit max_seq {self.stack.max_seq}")
            ids = torch.tensor(prompt, dtype=torch.int32, device=self.device)
            h = torch.empty((T, H), device=self.device, dtype=torch.float32)
            self._embed(ids, h)
            self._wait(st.send_work)
            st.send_work = None
            hdr[H_POS], hdr[H_STREAM], hdr[H_T], hdr[H_FLAGS] = 0, sid, T, FLAG_PREFILL | FLAG_RESET
            if self.runs[0].owner != 0:
                self._wait(self._send(st.msg, self.runs[0].owner))
                self._wait(self._send(h, self.runs[0].owner))
        for j, run in enumerate(self.runs):
            if run.owner != self.rank:
                continue
            if self.is_master and j == 0:
                self.stack.forward(h, run.layers, 0, session=sid)
                nxt = self._next(j)
                if nxt != self.rank:
                    self._wait(self._send(st.msg, nxt))
                    self._wait(self._send(h, nxt))
                continue
            self._wait(st.send_work)
            st.send_work = None
            self._recv(st.msg, self._prev(j))
            h = self._prefill_run(st, j)
        if not self.is_master:
            return None
        if self.runs[-1].owner != 0:
            self._recv(st.msg, self._final_src())
            h = torch.empty((int(hdr[H_T].item()), H), device=self.device, dtype=torch.float32)
            self._recv(h, self._final_src())
        hdr[H_FLAGS] = 0
        T = len(prompt)
        st.dev_pos = T
        if self.hip:
            b = st.bufs
            b.hist[:T].copy_(ids)
            b.hist_len.fill_(T)
            b.pos.fill_(T - 1)
            b.slot.zero_()
            self._logits(h[-1].contiguous(), b.logits)
            self._select_device(st)
            if self.sampler is not None:
                return self._host_sample_device(st)
            return int(b.tok.item())
        st.host_tokens = list(prompt)
        tok = self._select_host(st, self._logits(h[-1]))
        st.host_tokens.append(tok)
        st.host_pos = T
        st.hdr[H_POS] = T
        return tok

    def _prefill_run(self, st: _Stream, j: int) -> torch.Tensor:
        """Worker side of one prefill hop: the control message is already in st.msg."""
        H = self.cfg.hidden_size
        T, pos0, sid = int(st.hdr[H_T].item()), int(st.hdr[H_POS].item()), int(st.hdr[H_STREAM].item())
        h = torch.empty((T, H), device=self.device, dtype=torch.float32)
        self._recv(h, self._prev(j))
        if int(st.hdr[H_FLAGS].item()) & FLAG_RESET:
            self.stack.reset(sid)
        self.stack.forward(h, self.runs[j].layers, pos0, session=sid)
        st.dev_pos = pos0 + T
        nxt = self._next(j)
        if nxt != self.rank:
            self._wait(self._send(st.msg, nxt))
            self._wait(self._send(h, nxt))
        return h

    # ------------------------------------------------------------------ serving (control-gated)
    def ctrl_send(self, cmd: dict) -> None:
        """Master: one control message to every worker (host, gloo group)."""
        if self.ctrl is not None:
            dist.broadcast_object_list([cmd], src=0, group=self.ctrl)

    def _ctrl_recv(self) -> dict:
        box = [None]
        dist.broadcast_object_list(box, src=0, group=self.ctrl)
        return box[0]

    def serve(self) -> None:
        """Worker loop (CLI/API master on rank 0, stream 0): block on the host control
        channel, then run what the master announced — ``prefill`` (the [T, H] hops
        follow), ``decode n`` (n token replays: with ipc hops they are enqueued at
        once and the device-side receives pace them), ``stop``.  A worker never
        waits in a device-side receive for work that was not announced, so an idle
        server cannot hit the hop timeout."""
        if self.is_master:
            raise RuntimeError("serve() is the worker loop")
        st = self.streams[0]
        while True:
            cmd = self._ctrl_recv()
            op = cmd.get("op")
            if op == "stop":
                self.flush()
                if self.hop == "ipc" and self.hip:
                    torch.cuda.synchronize(self.device)
                    self.check_hops()
                return
            if op == "prefill":
                self.flush()
                if self.hop == "ipc" and self.hip:
                    torch.cuda.synchronize(self.device)
                    self.check_hops()
                self.prefill(0)
            elif op == "decode":
                st.dev_pos = int(cmd["pos"])
                self.decode(int(cmd["n"]))
            else:
                raise RuntimeError(f"unknown control message {cmd!r}")

    def decode_budget(self, sid: int = 0) -> int:
        """Decode steps that still fit the KV cache / token history of a stream."""
        return max(0, self.stack.max_seq - 1 - self.streams[sid].dev_pos)

    def generate(self, n: int, on_token=None, eos_ids=None, chunk: int | None = None) -> list[int]:
        """Master, after prefill(0, prompt): up to n more tokens of stream 0 (clamped to
        the cache), stopping at EOS.  Work is announced to the workers in chunks; the
        next chunk is announced before the current one is read back, so the ranks
        never idle between chunks.  Tokens are read back one replay behind (pinned
        ring + events); the at most two chunks enqueued past an EOS are discarded
        (the next prefill resets the stream)."""
        import collections
        if not self.is_master:
            raise RuntimeError("generate() runs on the master")
        st = self.streams[0]
        n = min(int(n), self.decode_budget(0))
        out: list[int] = []
        if n <= 0:
            return out
        ipc = self.hop == "ipc" and self.use_graph
        chunk = max(1, int(chunk or (16 if ipc else 1)))
        single = self.world == 1 or all(r.owner == 0 for r in self.runs)
        if ipc and self.hip and self.k == 1 and (st.sid, "tok") in st.graphs:
            return self._generate_native(st, n, on_token, eos_ids, chunk, single)
        if ipc and self.k > 1:
            # one ipc replay is k tokens: the announcements, hop counts and read-back
            # below count replays as tokens, so the ranks would fall out of step
            raise ValueError("generate() with ipc hops needs steps_per_graph == 1 "
                             f"(got {self.k}); use run_rounds() for k-token replays")
        base = int(st.bufs.hist_len.item()) if self.hip else 0
        ring = torch.empty(max(1, n), dtype=torch.int32, pin_memory=self.hip and
                           torch.cuda.is_available()) if self.hip else None
        pending: collections.deque = collections.deque()
        issued = 0
        self._events = []
        if self.hip:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
            self._events.append(ev0)

        def issue() -> None:
            nonlocal issued
            c = min(chunk, n - issued)
            if not single:
                self.ctrl_send({"op": "decode", "n": c, "pos": st.dev_pos})
            for _ in range(c):
                if ipc:
                    self._replay_ipc_token(st)
                else:
                    self._step_host(st, single)
                i = issued
                issued += 1
                if self.hip:
                    ring[i:i + 1].copy_(st.bufs.hist[base + i:base + i + 1], non_blocking=True)
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                    self._events.append(ev)
                    pending.append((i, ev))
                else:
                    pending.append((i, None))
        issue()
        stop = False
        while pending:
            if issued < n and len(pending) <= chunk and not stop:
                issue()
            i, ev = pending.popleft()
            if stop:
                continue
            if ev is not None:
                ev.synchronize()
                tok = int(ring[i].item())
            else:
                tok = st.host_tokens[-(issued - i)]
            out.append(tok)
            if on_token is not None:
                on_token(tok)
            if eos_ids and tok in eos_ids:
                stop = True
        if self.hip:
            torch.cuda.synchronize(self.device)
        self.check_hops()
        return out

    def _graph_set(self, st: "_Stream"):
        """This rank's token graphs of stream st as a native-loop GraphSet."""
        gs = getattr(st, "graph_set", None)
        graphs = st.graphs[(st.sid, "tok")]
        if gs is None or gs.graphs[-1] is not graphs[max(graphs)]:
            from ..ops import graph_loop as GL
            caps = sorted(graphs)
            idx = {id(graphs[c]): i for i, c in enumerate(caps)}
            gs = st.graph_set = GL.GraphSet([graphs[c] for c in caps],
                                            lambda t: idx[id(self._pick(graphs, t))],
                                            self.stack.max_seq)
        return gs

    def _generate_native(self, st: "_Stream", n: int, on_token, eos_ids, chunk: int,
                         single: bool) -> list[int]:
        """generate() with ipc hops: the native loop (csrc/driver/graph_loop.cpp)
        replays this rank's token graph, announces each chunk to the workers one chunk
        ahead (the control callback) and reads tokens back one replay behind."""
        from ..ops import graph_loop as GL
        pos0 = st.dev_pos

        def announce(first: int, count: int) -> None:
            if not single:
                self.ctrl_send({"op": "decode", "n": count, "pos": pos0 + first})

        res = GL.run(self._graph_set(st), k=1, n=n, pos=pos0, hist=st.bufs.hist,
                     base=int(st.bufs.hist_len.item()), eos_ids=eos_ids,
                     on_token=(lambda t: bool(on_token(t))) if on_token is not None else None,
                     announce=announce, chunk=chunk)
        st.dev_pos = res.pos
        self._native_step_ms = res.step_ms
        torch.cuda.synchronize(self.device)
        self.check_hops()
        return res.tokens

    def _step_host(self, st: "_Stream", single: bool) -> None:
        """One master token with host-issued hops (dist transport / no graphs)."""
        self._wait(st.send_work)
        st.send_work = None
        st.hdr[H_FLAGS] = 0
        self._replay(st, "first", lambda: self._body_first(st))
        if not single:
            self._wait(self._send(st.msg, self._first_dst()))
            self._worker_runs(st)
            self._wait(st.send_work)
            st.send_work = None
            self._recv(st.msg, self._final_src())
        self._replay(st, "last", lambda: self._body_last(st))
        st.dev_pos += 1

    def step(self, sid: int = 0) -> int:
        """Master: one decode step of one stream with host-issued hops; returns the token
        (tests and the dist transport; workers run decode(1) for it)."""
        st = self.streams[sid]
        if self.stack.max_seq - 1 - st.dev_pos <= 0:
            raise ValueError("KV cache full (max_seq)")
        self._step_host(st, self.world == 1 or all(r.owner == 0 for r in self.runs))
        if self.hip:
            if self.sampler is not None:
                return self._host_sample_device(st)
            return int(st.bufs.tok.item())
        return st.host_tokens[-1]

    def shutdown(self) -> None:
        """Master: tell every worker to leave serve()."""
        if not self.is_master or self.world == 1:
            return
        self.flush()
        self.ctrl_send({"op": "stop"})

    # ------------------------------------------------------------------ decode bodies
    def _body_first(self, st: _Stream) -> None:
        """Master: embed the stream's token (+ its run 0 layers if it owns run 0)."""
        if self.hip:
            from ..ops import hip as K
            K.embed(self.head.embed, st.bufs.tok, st.resid)
            if self.runs[0].owner == 0:
                self.stack.decode_step(st.bufs, self.runs[0].layers, st.sid)
        else:
            tok = torch.tensor([st.host_tokens[-1]], dtype=torch.int32, device=self.device)
            self._embed(tok, st.resid.view(1, -1))
            if self.runs[0].owner == 0:
                self.stack.forward(st.resid.view(1, -1), self.runs[0].layers, st.host_pos, st.sid)

    def _body_run(self, st: _Stream, j: int) -> None:
        if self.hip:
            self.stack.decode_step(st.bufs, self.runs[j].layers, st.sid)
        else:
            pos = int(st.hdr[H_POS].item())
            self.stack.forward(st.resid.view(1, -1), self.runs[j].layers, pos, st.sid)

    def _body_last(self, st: _Stream) -> None:
        """Master: (its last run if it owns it) + ln_f/lm_head + token selection."""
        last = len(self.runs) - 1
        if self.hip:
            if self.runs[last].owner == 0 and last > 0:
                self.stack.decode_step(st.bufs, self.runs[last].layers, st.sid)
            from ..ops import hip as K
            K.norm_gemv_f32(st.resid, self.head.norm, self.cfg.rms_norm_eps, self.head.lm_head,
                            st.bufs.logits)
            self._select_device(st)
        else:
            if self.runs[last].owner == 0 and last > 0:
                self.stack.forward(st.resid.view(1, -1), self.runs[last].layers, st.host_pos,
                                   st.sid)
            tok = self._select_host(st, self._logits(st.resid))
            st.host_tokens.append(tok)
            st.host_pos += 1
            st.hdr[H_POS] = st.host_pos

    # ------------------------------------------------------------------ graphs
    def _caps(self) -> list[int]:
        from ..ops import hip as K
        return K.attn_split_caps(self.stack.max_seq)

    def _capture_caps(self, fn) -> dict:
        """One graph of fn per attention split cap (position buckets)."""
        from ..ops import hip as K
        out = {}
        for cap in self._caps():
            g = torch.cuda.CUDAGraph()
            with K.attn_split_cap(cap), torch.cuda.graph(g):
                fn()
            out[cap] = g
        return out

    @staticmethod
    def _pick(graphs: dict, tk: int):
        """Smallest-cap graph whose split count covers live length tk (any cap is
        correct; a larger one only launches idle attention workgroups)."""
        from ..ops import hip as K
        need = K.attn_splits(tk)
        for cap in sorted(graphs):
            if cap >= need:
                return graphs[cap]
        return graphs[max(graphs)]

    def _replay(self, st: _Stream, key: str, fn) -> None:
        if not self.use_graph:
            fn()
            return
        gs = st.graphs.get(key)
        if gs is None:
            raise RuntimeError("capture() first")
        self._pick(gs, st.dev_pos + 2).replay()

    def _warm(self, st: _Stream, fn) -> None:
        """Run fn once outside capture on scratch state (the K/V row written is the
        cache's last one), then restore the stream's message and token state."""
        saved = st.msg.clone()
        st.hdr[H_POS] = self.stack.max_seq - 1
        keep = None
        if self.is_master:
            b = st.bufs
            keep = [t.clone() for t in (b.tok, b.hist, b.hist_len, b.slot)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        st.msg.copy_(saved)
        if keep is not None:
            for t, v in zip((b.tok, b.hist, b.hist_len, b.slot), keep):
                t.copy_(v)

    def capture(self) -> None:
        """Capture the decode graphs (one per body and attention split cap) — RCCL hops
        stay outside.  With ipc hops the receives/sends are inside the graphs: one
        graph per stream holding this rank's stages of `k` consecutive tokens
        (streams = 1), or one per (stream, stage) replayed stage-major so streams
        overlap (streams > 1)."""
        if not self.use_graph:
            return
        if self.hop == "ipc":
            self._capture_ipc()
            return
        for st in self.streams:
            for key, fn in self._bodies(st).items():
                self._warm(st, fn)
                st.graphs[key] = self._capture_caps(fn)
        torch.cuda.synchronize()

    def _capture_ipc(self) -> None:
        bodies = {}
        for st in self.streams:
            if len(self.streams) == 1:
                bodies[(st.sid, "tok")] = (st, lambda st=st: [self._ipc_token_body(st)
                                                              for _ in range(self.k)])
            else:
                for k in self._ipc_stages():
                    bodies[(st.sid, k)] = (st, lambda st=st, k=k: self._ipc_stage_body(st, k))
        # warm-up outside capture WITHOUT hops (a receive would wait on a peer that
        # is not sending), on scratch state that is restored afterwards
        self._skip_hops = True
        try:
            for key, (st, fn) in bodies.items():
                self._warm(st, (lambda st=st: self._ipc_token_body(st)) if len(self.streams) == 1
                           else fn)
        finally:
            self._skip_hops = False
        for key, (st, fn) in bodies.items():
            st.graphs[key] = self._capture_caps(fn)
        torch.cuda.synchronize()

    def _replay_ipc_token(self, st: _Stream) -> None:
        """This rank's part of one token of stream st (streams = 1, k = 1 graphs)."""
        self._pick(st.graphs[(st.sid, "tok")], st.dev_pos + self.k + 1).replay()
        st.dev_pos += self.k

    def _decode_ipc(self, rounds: int) -> None:
        """Every rank enqueues its graphs for `rounds` tokens; the hops synchronise
        the ranks on the device.  The master records one event per replay."""
        if len(self.streams) == 1:
            st = self.streams[0]
            if not self.is_master:  # worker: native enqueue of every replay
                from ..ops import graph_loop as GL
                st.dev_pos = GL.run(self._graph_set(st), k=self.k, n=rounds, pos=st.dev_pos).pos
                return
            for _ in range(rounds // self.k):
                self._replay_ipc_token(st)
                if self.is_master:
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                    self._events.append(ev)
            return
        stages = self._ipc_stages()
        for _ in range(rounds):
            for k in stages:
                for st in self.streams:
                    self._pick(st.graphs[(st.sid, k)], st.dev_pos + 2).replay()
            for st in self.streams:
                st.dev_pos += 1
            if self.is_master:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self._events.append(ev)

    def step_times_ms(self) -> list[float]:
        """Master: per-replay device intervals recorded by the last ipc decode()
        (per token when streams = 1 and k = 1; otherwise per round / per k tokens)."""
        ev = self._events
        return [a.elapsed_time(b) for a, b in zip(ev, ev[1:])]

    def _bodies(self, st: _Stream) -> dict:
        out = {}
        if self.is_master:
            out["first"] = lambda st=st: self._body_first(st)
            out["last"] = lambda st=st: self._body_last(st)
        for j in self.my_runs:
            if self.is_master and (j == 0 or j == len(self.runs) - 1):
                continue
            out[f"run{j}"] = lambda st=st, j=j: self._body_run(st, j)
        return out

    # ------------------------------------------------------------------ decode loop
    def decode(self, rounds: int) -> None:
        """Every stream generates `rounds` tokens (ignoring EOS); every rank calls it
        with the same `rounds` (the bench; serve() for workers)."""
        if rounds <= 0:
            return
        for st in self.streams:
            if st.dev_pos + rounds > self.stack.max_seq - 1:
                raise ValueError(f"decode of {rounds} tokens from position {st.dev_pos} "
                                 f"overruns max_seq {self.stack.max_seq}")
        if self.hop == "ipc":
            if len(self.streams) == 1 and rounds % self.k:
                raise ValueError(f"rounds ({rounds}) must be a multiple of steps_per_graph "
                                 f"({self.k})")
            self._events = []
            if self.is_master:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self._events.append(ev)
            self._decode_ipc(rounds)
            return
        single = self.world == 1 or all(r.owner == 0 for r in self.runs)
        self._events = []
        timed = self.is_master and self.hip

        def mark():
            if timed:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self._events.append(ev)
        mark()
        for k in range(rounds):
            if k > 0:
                mark()
            for st in self.streams:
                if self.is_master:
                    if single:
                        self._replay(st, "first", lambda: self._body_first(st))
                        self._replay(st, "last", lambda: self._body_last(st))
                        st.dev_pos += 1
                        continue
                    self._wait(st.send_work)
                    if k > 0:
                        self._recv(st.msg, self._final_src())
                        self._replay(st, "last", lambda: self._body_last(st))
                        st.dev_pos += 1
                    self._replay(st, "first", lambda: self._body_first(st))
                    st.send_work = self._send(st.msg, self._first_dst())
                self._worker_runs(st)
                if not self.is_master:
                    st.dev_pos += 1
        if self.is_master and not single:
            for st in self.streams:
                self._wait(st.send_work)
                st.send_work = None
                self._recv(st.msg, self._final_src())
                self._replay(st, "last", lambda: self._body_last(st))
                st.dev_pos += 1
        mark()

    def _worker_runs(self, st: _Stream) -> None:
        last = len(self.runs) - 1
        for j in self.my_runs:
            if self.is_master and (j == 0 or j == last):
                continue
            self._wait(st.send_work)
            self._recv(st.msg, self._prev(j))
            self._replay(st, f"run{j}", lambda j=j: self._body_run(st, j))
            st.send_work = self._send(st.msg, self._next(j))

    def flush(self) -> None:
        for st in self.streams:
            self._wait(st.send_work)
            st.send_work = None

    def tokens(self, sid: int) -> list[int]:
        """Master: full token history (prompt + generated) of a stream."""
        st = self.streams[sid]
        if self.hip:
            n = int(st.bufs.hist_len.item())
            return st.bufs.hist[:n].tolist()
        return list(st.host_tokens)
