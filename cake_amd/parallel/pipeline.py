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
        self.graphs: dict[str, torch.cuda.CUDAGraph] = {}
        self.send_work = None
        self.host_tokens: list[int] = []   # torch backend bookkeeping (master)
        self.host_pos = 0


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
            K.norm_gemv_f32(st.resid, self.head.norm, self.cfg.rms_norm_eps, self.head.lm_head,
                            st.bufs.logits)
            self._select_device(st)
        else:
            self.stack.decode_step(st.bufs, self.runs[k - 1].layers, st.sid)
        if k < R + 1 and self._recv_point(k + 1) and not self._skip_hops:
            self._ipc_send(st, k + 1)

    def _ipc_token_body(self, st: "_Stream") -> None:
        for k in self._ipc_stages():
            self._ipc_stage_body(st, k)

    def check_hops(self) -> None:
        """Raise if any device-side receive timed out (a peer stopped sending)."""
        if self.hop == "ipc" and int(self._err.item()) != 0:
            raise RuntimeError(f"rank {self.rank}: a pipeline hop timed out "
                               f"(CAKE_HOP_TIMEOUT={os.environ.get('CAKE_HOP_TIMEOUT', '60')} s)")

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
        nxt = self._next(j)
        if nxt != self.rank:
            self._wait(self._send(st.msg, nxt))
            self._wait(self._send(h, nxt))
        return h

    # ------------------------------------------------------------------ serving (message-driven)
    def serve(self) -> None:
        """Worker loop for interactive use (CLI/API master on rank 0, one stream):
        every hop starts with the stream's message; its header says PREFILL (a
        [T, H] block follows), STOP (forward it and return) or decode."""
        if self.is_master:
            raise RuntimeError("serve() is the worker loop")
        st = self.streams[0]
        runs = [j for j in self.my_runs]
        while True:
            stopped = False
            for j in runs:
                self._wait(st.send_work)
                st.send_work = None
                self._recv(st.msg, self._prev(j))
                flags = int(st.hdr[H_FLAGS].item())
                if flags & FLAG_STOP:
                    self._wait(self._send(st.msg, self._next(j)))
                    stopped = True
                    continue
                if flags & FLAG_PREFILL:
                    self._prefill_run(st, j)
                    continue
                self._replay(st, f"run{j}", lambda j=j: self._body_run(st, j))
                st.send_work = self._send(st.msg, self._next(j))
            if stopped:
                self.flush()
                return

    def step(self, sid: int = 0) -> int:
        """Master: one decode step of one stream; returns the new token id."""
        st = self.streams[sid]
        single = self.world == 1 or all(r.owner == 0 for r in self.runs)
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
        if self.hip:
            if self.sampler is not None:
                return self._host_sample_device(st)
            return int(st.bufs.tok.item())
        return st.host_tokens[-1]

    def shutdown(self) -> None:
        """Master: send STOP along the chain and wait for it to come back."""
        if not self.is_master or self.world == 1 or all(r.owner == 0 for r in self.runs):
            return
        st = self.streams[0]
        self._wait(st.send_work)
        st.send_work = None
        st.hdr[H_FLAGS] = FLAG_STOP
        self._wait(self._send(st.msg, self._first_dst()))
        for j in self.my_runs:   # master-owned middle runs see STOP too
            if j in (0, len(self.runs) - 1):
                continue
            self._recv(st.msg, self._prev(j))
            self._wait(self._send(st.msg, self._next(j)))
        self._recv(st.msg, self._final_src())

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

    def _replay(self, st: _Stream, key: str, fn) -> None:
        if not self.use_graph:
            fn()
            return
        g = st.graphs.get(key)
        if g is None:
            raise RuntimeError("capture() first")
        g.replay()

    def capture(self) -> None:
        """Capture one hipGraph per (stream, body) — RCCL hops stay outside.  With ipc
        hops the receives/sends are inside the graphs: one graph per stream holding
        this rank's stages of `k` consecutive tokens (streams = 1), or one per
        (stream, stage) replayed stage-major so streams overlap (streams > 1)."""
        if not self.use_graph:
            return
        if self.hop == "ipc":
            self._capture_ipc()
            return
        for st in self.streams:
            bodies = self._bodies(st)
            for key, fn in bodies.items():
                # warm-up on a scratch copy of the state the body mutates; the
                # warm-up writes K/V at a scratch position (last cache row) so
                # the prefilled rows are untouched
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
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    fn()
                st.graphs[key] = g
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
                saved = st.msg.clone()
                st.hdr[H_POS] = self.stack.max_seq - 1
                keep = None
                if self.is_master:
                    b = st.bufs
                    keep = [t.clone() for t in (b.tok, b.hist, b.hist_len, b.slot)]
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    if len(self.streams) == 1:
                        self._ipc_token_body(st)
                    else:
                        fn()
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                st.msg.copy_(saved)
                if keep is not None:
                    for t, v in zip((b.tok, b.hist, b.hist_len, b.slot), keep):
                        t.copy_(v)
        finally:
            self._skip_hops = False
        for key, (st, fn) in bodies.items():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            st.graphs[key] = g
        torch.cuda.synchronize()

    def _decode_ipc(self, rounds: int) -> None:
        """Every rank enqueues its graphs for `rounds` tokens; the hops synchronise
        the ranks on the device.  The master records one event per replay."""
        if len(self.streams) == 1:
            st = self.streams[0]
            g = st.graphs[(st.sid, "tok")]
            for _ in range(-(-rounds // self.k)):
                g.replay()
                if self.is_master:
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record()
                    self._events.append(ev)
            return
        stages = self._ipc_stages()
        for _ in range(rounds):
            for k in stages:
                for st in self.streams:
                    st.graphs[(st.sid, k)].replay()
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
        """Every stream generates `rounds` tokens (ignoring EOS)."""
        if self.hop == "ipc":
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
                        continue
                    self._wait(st.send_work)
                    if k > 0:
                        self._recv(st.msg, self._final_src())
                        self._replay(st, "last", lambda: self._body_last(st))
                    self._replay(st, "first", lambda: self._body_first(st))
                    st.send_work = self._send(st.msg, self._first_dst())
                self._worker_runs(st)
        if self.is_master and not single:
            for st in self.streams:
                self._wait(st.send_work)
                st.send_work = None
                self._recv(st.msg, self._final_src())
                self._replay(st, "last", lambda: self._body_last(st))
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
