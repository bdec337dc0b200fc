"""Transformer-block execution: a rank's local layers + their KV cache.

A :class:`LayerStack` is the MI355X-native counterpart of the reference's
per-layer ``Transformer`` forwarders (cake-core/src/models/llama3/transformer.rs)
plus the KV part of ``Cache`` (cache.rs:93-135).  Both the master (layers not
assigned to any worker) and each worker own one.

Two execution backends share the same weights and cache layout:

* ``hip``   — gfx950 kernels (:mod:`cake_amd.ops.hip`).  Decode (T=1) runs five
  fused launches per layer with the position read from device memory, so a
  whole token step is hipGraph-capturable; prefill (T>1) runs the projections
  on our MFMA GEMM (gemm.hip; residual / SwiGLU in its epilogues) plus the
  RoPE/KV-write and MFMA flash-attention kernels.
* ``torch`` — the Appendix-D reference math in PyTorch (CPU mode ``--cpu``,
  f32 dtype, and the oracle in tests).

KV cache: one preallocated ``[n_local, nkv, max_seq, hd]`` K and V tensor per
session (SURVEY Appendix E Q2 — no ``Tensor::cat`` growth).  Sessions isolate
concurrent masters on one worker (worker.rs:52-72) and are reset explicitly
(fixes Appendix E Q7).
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import torch

from ...ops import reference as R
from .config import LlamaConfig
from .weights import BlockWeights


class KVCache:
    def __init__(self, n_layers: int, cfg: LlamaConfig, max_seq: int, device, dtype):
        shape = (n_layers, cfg.num_key_value_heads, max_seq, cfg.head_dim)
        self.k = torch.zeros(shape, device=device, dtype=dtype)
        self.v = torch.zeros(shape, device=device, dtype=dtype)
        self.max_seq = max_seq
        self.length = 0  # number of valid positions (host bookkeeping)

    def clear(self) -> None:
        self.length = 0


class DecodeBuffers:
    """Device-resident state of a batch-1 decode step (graph-stable addresses)."""

    def __init__(self, cfg: LlamaConfig, max_seq: int, device, dtype, with_head: bool,
                 resid: torch.Tensor | None = None, pos: torch.Tensor | None = None):
        H, I, hd, nh = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim, cfg.num_attention_heads
        f32, i32 = torch.float32, torch.int32
        self.resid = torch.zeros(H, device=device, dtype=f32) if resid is None else resid
        self.q = torch.zeros(nh * hd, device=device, dtype=f32)
        self.attn_out = torch.zeros(nh * hd, device=device, dtype=dtype)
        self.act = torch.zeros(I, device=device, dtype=dtype)
        # <= 64 splits per head, 8-byte granules (attention.hip); tickets: [2 nkv] + the
        # merge's error word (+1 pad)
        self.part = torch.zeros(2 * nh * 64 * (hd + 2), device=device, dtype=f32)
        self.tickets = torch.zeros(2 * cfg.num_key_value_heads + 2, device=device, dtype=i32)
        # fused attention + o_proj (attn_oproj.hip): per-group partial rows, row-block
        # arrival tickets (zeroed once, re-armed by the kernel)
        nkv = cfg.num_key_value_heads
        self.ao_ws = torch.zeros(2 * nkv * H, device=device, dtype=f32)
        self.ao_tickets = torch.zeros(2 * (H // 32) + 2 * nkv + 2, device=device, dtype=i32)
        self.pos = torch.zeros(1, device=device, dtype=i32) if pos is None else pos
        if with_head:
            self.logits = torch.zeros(cfg.vocab_size, device=device, dtype=f32)
            self.tok = torch.zeros(1, device=device, dtype=i32)
            self.hist = torch.zeros(max_seq, device=device, dtype=i32)
            self.hist_len = torch.zeros(1, device=device, dtype=i32)
            self.slot = torch.zeros(1, device=device, dtype=torch.int64)
            self.thr = torch.zeros(1, device=device, dtype=torch.int32)  # top-k/p threshold
            self.sel_ticket = torch.zeros(1, device=device, dtype=i32)  # fused head_select


class LayerStack:
    def __init__(self, cfg: LlamaConfig, weights: dict[int, BlockWeights], device, dtype,
                 max_seq: int, backend: str, max_sessions: int = 8):
        if backend not in ("hip", "torch"):
            raise ValueError(f"unknown backend {backend}")
        if backend == "hip" and dtype not in (torch.bfloat16, torch.float16):
            raise ValueError("hip backend needs bf16/f16 weights (use torch backend for f32)")
        self.cfg = cfg
        self.weights = dict(sorted(weights.items()))
        self.slot_of = {li: i for i, li in enumerate(self.weights)}
        self.device = torch.device(device)
        self.dtype = dtype
        self.max_seq = max_seq
        self.backend = backend
        self.max_sessions = max_sessions
        self.inv_freq = R.inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling).to(self.device)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self._sessions: OrderedDict[int, KVCache] = OrderedDict()
        self._decode_bufs: DecodeBuffers | None = None
        self._hostpos_bufs: DecodeBuffers | None = None
        self.step_graphs = False  # T = 1 forward() as graph replays (worker serving)
        self._step_graph_cache: dict = {}
        # persistent decode (decode_mk.hip): one launch per token step instead of five
        # per layer; CAKE_MK=0 keeps the per-layer launches
        self.use_mk = os.environ.get("CAKE_MK", "0") != "0" and backend == "hip"
        self._mk_ok: bool | None = None
        self._mk_tables: dict = {}

    # ------------------------------------------------------------------ sessions
    def cache(self, session: int = 0) -> KVCache:
        kv = self._sessions.get(session)
        if kv is None:
            while len(self._sessions) >= self.max_sessions:
                old, _ = self._sessions.popitem(last=False)
                self._drop_step_graphs(old)  # their graphs point at the evicted cache
                for k in [k for k in self._mk_tables if k[0] == old]:
                    del self._mk_tables[k]
            kv = KVCache(len(self.weights), self.cfg, self.max_seq, self.device, self.dtype)
            self._sessions[session] = kv
        else:
            self._sessions.move_to_end(session)
        return kv

    def reset(self, session: int | None = None) -> None:
        if session is None:
            for kv in self._sessions.values():
                kv.clear()
        elif session in self._sessions:
            self._sessions[session].clear()

    def drop(self, session: int) -> None:
        self._sessions.pop(session, None)
        self._drop_step_graphs(session)
        for k in [k for k in self._mk_tables if k[0] == session]:
            del self._mk_tables[k]

    @property
    def layer_ids(self) -> list[int]:
        return list(self.weights)

    def decode_buffers(self, with_head: bool = False) -> DecodeBuffers:
        if self._decode_bufs is None or (with_head and not hasattr(self._decode_bufs, "logits")):
            self._decode_bufs = DecodeBuffers(self.cfg, self.max_seq, self.device, self.dtype,
                                              with_head)
        return self._decode_bufs

    # ------------------------------------------------------------------ forward
    def forward(self, hidden: torch.Tensor, layers: list[int], pos0: int,
                session: int = 0) -> torch.Tensor:
        """Run `layers` (in order) over hidden [T, H] f32 at positions pos0.., in place."""
        if hidden.dtype != torch.float32 or hidden.dim() != 2:
            raise ValueError("hidden must be f32 [T, H]")
        T = hidden.shape[0]
        kv = self.cache(session)
        if pos0 + T > self.max_seq:
            raise ValueError(f"sequence length {pos0 + T} exceeds max_seq {self.max_seq}")
        if self.backend == "hip" and T == 1 and self.step_graphs and hidden.is_cuda:
            self._decode_graph(hidden, layers, pos0, session)
            kv.length = max(kv.length, pos0 + 1)
            return hidden
        for li in layers:
            w = self.weights[li]
            s = self.slot_of[li]
            if self.backend == "hip":
                if T == 1:
                    self._decode_hip_hostpos(hidden, w, kv.k[s], kv.v[s], pos0)
                else:
                    self._prefill_hip(hidden, w, kv.k[s], kv.v[s], pos0)
            else:
                self._block_torch(hidden, w, kv.k[s], kv.v[s], pos0)
        kv.length = max(kv.length, pos0 + T)
        return hidden

    def mk_enabled(self) -> bool:
        """Whether decode steps run as ONE persistent launch (decode_mk.hip)."""
        if not self.use_mk:
            return False
        if self._mk_ok is None:
            from ...ops import hip as K
            cfg = self.cfg
            self._mk_ok = bool(torch.cuda.is_available() and self.device.type == "cuda"
                               and K.mk_supported(cfg.hidden_size, cfg.intermediate_size,
                                                  cfg.num_attention_heads,
                                                  cfg.num_key_value_heads, cfg.head_dim))
        return self._mk_ok

    def mk_table(self, layers: list[int], session: int = 0) -> torch.Tensor:
        """int64 [len(layers), 8] device pointer table of the persistent decode:
        ln1, wqkv, wo, ln2, wgu, wd and the session's K/V cache of each layer."""
        key = (session, tuple(layers))
        t = self._mk_tables.get(key)
        if t is None:
            kv = self.cache(session)
            rows = []
            for li in layers:
                w, s = self.weights[li], self.slot_of[li]
                rows.append([w.ln1.data_ptr(), w.wqkv.data_ptr(), w.wo.data_ptr(),
                             w.ln2.data_ptr(), w.wgu.data_ptr(), w.wd.data_ptr(),
                             kv.k[s].data_ptr(), kv.v[s].data_ptr()])
            t = torch.tensor(rows, dtype=torch.int64).to(self.device)
            self._mk_tables[key] = t
        return t

    def mk_workspace(self, bufs: DecodeBuffers) -> tuple[torch.Tensor, torch.Tensor]:
        """The persistent decode's granule workspace and control words (zeroed once;
        sized for every local layer, so any run of them can use it)."""
        if getattr(bufs, "mk_gran", None) is None:
            from ...ops import hip as K
            cfg = self.cfg
            words = len(self.weights) * K.mk_gstride(cfg.hidden_size, cfg.intermediate_size,
                                                     cfg.num_attention_heads,
                                                     cfg.num_key_value_heads, cfg.head_dim)
            bufs.mk_gran = torch.zeros(words, dtype=torch.int64, device=self.device)
            bufs.mk_ctl = torch.zeros(K.MK_CTL_WORDS, dtype=torch.int32, device=self.device)
        return bufs.mk_gran, bufs.mk_ctl

    def mk_check(self, bufs: DecodeBuffers) -> None:
        """Raise if a decode launch gave up waiting in one of its bounded spins: the
        persistent decode's hand-offs, or the split-K attention merge (host sync)."""
        from ...ops import hip as K
        if K.attn_error(bufs.tickets):
            K.attn_clear_error(bufs.tickets)
            raise RuntimeError("decode attention: a split merge timed out waiting for its "
                               "partials; outputs of that launch are invalid")
        ctl = getattr(bufs, "mk_ctl", None)
        if ctl is None:
            return
        site = K.mk_error(ctl)
        if site:
            ctl.zero_()
            raise RuntimeError(f"persistent decode: a hand-off timed out (site {site}); "
                               "outputs of that launch are invalid")

    def attn_oproj_ok(self) -> bool:
        """The fused decode attention + o_proj launch is enabled (opt-in, CAKE_ATTN_OPROJ=1:
        slower than the unfused pair on MI355X, profiles/r5_attn_oproj_ab.md) and covers
        this stack's shapes."""
        if self.backend != "hip" or os.environ.get("CAKE_ATTN_OPROJ", "0") != "1":
            return False
        from ...ops import hip as K
        c = self.cfg
        return K.attn_oproj_supported(c.num_attention_heads, c.num_key_value_heads,
                                      c.head_dim, c.hidden_size)

    def decode_step(self, bufs: DecodeBuffers, layers: list[int], session: int = 0,
                    fused: bool | None = None) -> None:
        """Graph-capturable T=1 step over bufs.resid at device position bufs.pos (hip only):
        five launches per layer (QKV+RoPE+KV write, attention, o_proj+residual,
        norm+gate/up+SwiGLU, down_proj+residual), or four with attention and o_proj as
        one launch when `fused` (default: inside K.attn_oproj_fused(), i.e. the
        short-context graph bucket; the caller guarantees one attention split); or the
        experimental persistent launch (decode_mk.hip, CAKE_MK=1, if built)."""
        from ...ops import hip as K
        cfg = self.cfg
        if layers and self.mk_enabled():
            gran, ctl = self.mk_workspace(bufs)
            K.mk_decode(self.dtype, self.mk_table(layers, session), len(layers), cfg.hidden_size,
                        cfg.intermediate_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                        cfg.head_dim, self.max_seq, cfg.rms_norm_eps, self.scale, self.inv_freq,
                        bufs.pos, bufs.resid, gran, ctl)
            return
        kv = self.cache(session)
        if fused is None:
            fused = K.attn_oproj_active()
        fused = fused and self.attn_oproj_ok()
        for li in layers:
            w = self.weights[li]
            s = self.slot_of[li]
            kc, vc = kv.k[s], kv.v[s]
            K.qkv_rope(bufs.resid, w.ln1, cfg.rms_norm_eps, w.wq, w.wk, w.wv,
                       self.inv_freq, bufs.pos, bufs.q, kc, vc)
            if fused:
                K.attn_oproj(bufs.q, kc, vc, bufs.pos, self.scale, w.wo, bufs.resid, True,
                             bufs.ao_ws, bufs.ao_tickets, bufs.tickets)
            else:
                K.attn_decode(bufs.q, kc, vc, bufs.pos, self.scale, bufs.part, bufs.tickets,
                              bufs.attn_out)
                K.gemv(bufs.attn_out, w.wo, bufs.resid, accumulate=True)
            K.swiglu(bufs.resid, w.ln2, cfg.rms_norm_eps, w.wg, w.wu, bufs.act)
            K.gemv(bufs.act, w.wd, bufs.resid, accumulate=True)

    # ------------------------------------------------------------------ hip paths
    def _decode_graph(self, hidden, layers: list[int], pos0: int, session: int) -> None:
        """T = 1 over a run of layers as ONE graph replay (worker serving path): the
        first request of a (session, run, attention split cap) runs eagerly and
        captures the step; later ones copy the hidden state and position in, replay,
        copy the state out.  The position is known on the host here, so the graph is
        the one of the smallest split cap covering the live length (position
        buckets, as DeviceDecoder.capture)."""
        from ...ops import hip as K
        full = K.attn_max_split(self.max_seq)
        need = K.attn_splits(pos0 + 1)
        cap = next((c for c in (8, 16, 32, 64) if c >= min(need, full)), 64)
        cap = min(cap, full)
        if K.attn_oproj_short(pos0) and self.attn_oproj_ok():
            cap = 1  # one split: attention and o_proj as one launch per layer
        key = (session, tuple(layers), cap)
        ent = self._step_graph_cache.get(key)
        if ent is None:
            bufs = next((b for (s, l, _), (_, b) in self._step_graph_cache.items()
                         if s == session and l == key[1]), None)
            if bufs is None:
                bufs = DecodeBuffers(self.cfg, self.max_seq, self.device, self.dtype,
                                     with_head=False)
            bufs.pos.fill_(pos0)
            bufs.resid.copy_(hidden[0])
            self.decode_step(bufs, layers, session, fused=cap == 1)
            hidden[0].copy_(bufs.resid)
            g = torch.cuda.CUDAGraph()
            with K.attn_split_cap(cap if cap != 1 else full), K.attn_oproj_fused(cap == 1), \
                    torch.cuda.graph(g):  # records only
                self.decode_step(bufs, layers, session)
            self._step_graph_cache[key] = (g, bufs)
            return
        g, bufs = ent
        bufs.pos.fill_(pos0)
        bufs.resid.copy_(hidden[0])
        g.replay()
        hidden[0].copy_(bufs.resid)

    def _drop_step_graphs(self, session: int) -> None:
        for k in [k for k in self._step_graph_cache if k[0] == session]:
            del self._step_graph_cache[k]

    def _decode_hip_hostpos(self, hidden, w, kc, vc, pos0):
        if self._hostpos_bufs is None:
            self._hostpos_bufs = DecodeBuffers(self.cfg, self.max_seq, self.device, self.dtype,
                                               with_head=False)
        bufs = self._hostpos_bufs
        bufs.pos.fill_(pos0)
        bufs.resid.copy_(hidden[0])
        from ...ops import hip as K
        cfg = self.cfg
        K.qkv_rope(bufs.resid, w.ln1, cfg.rms_norm_eps, w.wq, w.wk, w.wv, self.inv_freq,
                   bufs.pos, bufs.q, kc, vc)
        if K.attn_oproj_short(pos0) and self.attn_oproj_ok():
            K.attn_oproj(bufs.q, kc, vc, bufs.pos, self.scale, w.wo, bufs.resid, True,
                         bufs.ao_ws, bufs.ao_tickets, bufs.tickets)
        else:
            K.attn_decode(bufs.q, kc, vc, bufs.pos, self.scale, bufs.part, bufs.tickets,
                          bufs.attn_out)
            K.gemv(bufs.attn_out, w.wo, bufs.resid, accumulate=True)
        K.swiglu(bufs.resid, w.ln2, cfg.rms_norm_eps, w.wg, w.wu, bufs.act)
        K.gemv(bufs.act, w.wd, bufs.resid, accumulate=True)
        hidden[0].copy_(bufs.resid)

    def _prefill_hip(self, hidden, w, kc, vc, pos0):
        """T > 1 block on MFMA GEMMs (gemm.hip) with fused epilogues: q|k|v in one
        GEMM, o_proj and down_proj accumulate into the f32 residual stream, the
        gate|up GEMM applies SwiGLU in its epilogue."""
        from ...ops import gemm as G
        from ...ops import hip as K
        cfg = self.cfg
        T, H = hidden.shape
        x = torch.empty((T, H), device=hidden.device, dtype=self.dtype)
        K.rmsnorm(hidden, w.ln1, cfg.rms_norm_eps, x)
        nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        nq, nk = nh * hd, nkv * hd
        qkv = G.linear(x, w.wqkv)  # one GEMM for q|k|v
        q, k, v = qkv[:, :nq], qkv[:, nq:nq + nk], qkv[:, nq + nk:]
        K.rope_kv(q, k, v, self.inv_freq, pos0, kc, vc)
        att = torch.empty((T, nq), device=hidden.device, dtype=self.dtype)
        Tk = pos0 + T
        K.flash_attn(q.view(1, T, nh, hd).transpose(1, 2), kc[None, :, :Tk], vc[None, :, :Tk],
                     att.view(1, T, nh, hd).transpose(1, 2), self.scale, causal=True, pos0=pos0)
        G.linear(att, w.wo, epi="resid32", resid=hidden)      # hidden += att @ wo^T
        K.rmsnorm(hidden, w.ln2, cfg.rms_norm_eps, x)
        act = G.linear(x, w.wgu, epi="swiglu")                # silu(x wg^T) * (x wu^T)
        G.linear(act, w.wd, epi="resid32", resid=hidden)      # hidden += act @ wd^T

    # ------------------------------------------------------------------ torch path
    def _block_torch(self, hidden, w, kc, vc, pos0):
        cfg = self.cfg
        T = hidden.shape[0]
        nh, nkv, hd = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        dt = self.dtype
        positions = torch.arange(pos0, pos0 + T, device=hidden.device)
        x = R.rms_norm(hidden, w.ln1, cfg.rms_norm_eps).to(dt)
        q = (x @ w.wq.t()).view(T, nh, hd)
        k = (x @ w.wk.t()).view(T, nkv, hd)
        v = (x @ w.wv.t()).view(T, nkv, hd)
        q = R.rope(q, positions, self.inv_freq).to(dt)
        k = R.rope(k, positions, self.inv_freq).to(dt)
        kc[:, pos0:pos0 + T] = k.transpose(0, 1)
        vc[:, pos0:pos0 + T] = v.to(dt).transpose(0, 1)
        Tk = pos0 + T
        att = R.attention(q, kc[:, :Tk].transpose(0, 1), vc[:, :Tk].transpose(0, 1), pos0)
        att = att.to(dt).reshape(T, nh * hd)
        hidden += (att @ w.wo.t()).float()
        x2 = R.rms_norm(hidden, w.ln2, cfg.rms_norm_eps).to(dt)
        act = R.silu_mul(x2 @ w.wg.t(), x2 @ w.wu.t()).to(dt)
        hidden += (act @ w.wd.t()).float()
