"""Master-side Llama-3 model: embedding → placed blocks → ln_f → lm_head.

Counterpart of ``LLama::forward`` (cake-core/src/models/llama3/llama.rs:72-138).
Blocks are placed per the topology: a layer named on a worker is reached
through a remote :class:`~cake_amd.parallel.forwarder.Forwarder`; every other
layer runs in this process's :class:`LayerStack`.  Consecutive layers with the
same owner form one *run* and cost one hop (contiguous-block batching,
llama.rs:95-114) — planned once at load time by :func:`plan_runs`.

For the all-local HIP case, :class:`DeviceDecoder` captures the whole decode
step (embedding, 32/80 layers, ln_f + lm_head, repeat penalty, argmax, next
token/position bookkeeping) into ONE hipGraph; the host reads 4 bytes per token,
one step behind the GPU.
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field

import torch

from ...ops import reference as R
from .blocks import DecodeBuffers, LayerStack
from .config import LlamaConfig
from .weights import HeadWeights, layer_name


@dataclass
class Run:
    ident: str                 # "local" or the worker identity
    layers: list[int]
    forwarder: object | None = None   # parallel.forwarder.Forwarder for remote runs

    @property
    def local(self) -> bool:
        return self.ident == "local"


def plan_runs(num_layers: int, remote: dict[int, object]) -> list[Run]:
    """Group consecutive layers with equal owner identity (llama.rs:95-114)."""
    runs: list[Run] = []
    for li in range(num_layers):
        fwd = remote.get(li)
        ident = "local" if fwd is None else fwd.ident()
        if runs and runs[-1].ident == ident:
            runs[-1].layers.append(li)
        else:
            runs.append(Run(ident=ident, layers=[li], forwarder=fwd))
    return runs


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, head: HeadWeights, stack: LayerStack,
                 remote: dict[int, object] | None = None):
        self.cfg = cfg
        self.head = head
        self.stack = stack
        self.remote = dict(remote or {})
        self.runs = plan_runs(cfg.num_hidden_layers, self.remote)
        missing = [li for r in self.runs if r.local for li in r.layers if li not in stack.weights]
        if missing:
            raise ValueError(f"local layers without weights: {missing[:8]}")
        self.device = stack.device
        self.dtype = stack.dtype
        self.backend = stack.backend
        self.session = 0

    @property
    def all_local(self) -> bool:
        return all(r.local for r in self.runs)

    # ------------------------------------------------------------------ generic path
    def embed(self, tokens: list[int]) -> torch.Tensor:
        ids = torch.tensor(tokens, dtype=torch.int32, device=self.device)
        if self.backend == "hip":
            from ...ops import hip as K
            out = torch.empty((len(tokens), self.cfg.hidden_size), device=self.device,
                              dtype=torch.float32)
            K.embed(self.head.embed, ids, out)
            return out
        return self.head.embed[ids.long()].float()

    def forward_hidden(self, hidden: torch.Tensor, pos0: int) -> torch.Tensor:
        for run in self.runs:
            if run.local:
                self.stack.forward(hidden, run.layers, pos0, self.session)
            else:
                batch = [(layer_name(li), pos0, li) for li in run.layers]
                hidden = run.forwarder.forward_batch(hidden, batch, self.session)
                if hidden.device != self.device:
                    hidden = hidden.to(self.device)
                hidden = hidden.float().contiguous()
        return hidden

    def head_logits(self, last: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """ln_f + lm_head on one f32 row -> f32 logits (llama.rs:119-137)."""
        if self.backend == "hip":
            from ...ops import hip as K
            if out is None:
                out = torch.empty(self.cfg.vocab_size, device=self.device, dtype=torch.float32)
            K.norm_gemv_f32(last.contiguous(), self.head.norm, self.cfg.rms_norm_eps,
                            self.head.lm_head, out)
            return out
        x = R.rms_norm(last, self.head.norm, self.cfg.rms_norm_eps).to(self.dtype)
        return (x @ self.head.lm_head.t()).float()

    def forward(self, tokens: list[int], pos0: int) -> torch.Tensor:
        """Logits (f32 [V]) of the last of `tokens`, fed at positions pos0.."""
        h = self.embed(tokens)
        h = self.forward_hidden(h, pos0)
        return self.head_logits(h[-1])

    def reset(self) -> None:
        self.stack.reset(self.session)
        for run in self.runs:
            if not run.local and hasattr(run.forwarder, "reset"):
                run.forwarder.reset(self.session)


@dataclass
class _Pending:
    event: torch.cuda.Event
    host: torch.Tensor
    t_issue: float = 0.0
    extra: dict = field(default_factory=dict)


class DeviceDecoder:
    """Whole-step hipGraph decoder for an all-local model on the HIP backend.

    Device state (DecodeBuffers): tok, pos, hist, hist_len, slot.  A step:
    embed(tok) → layers(pos) → ln_f/lm_head → [repeat penalty] → token
    selection → finalize (tok ← selected, hist.append, pos += 1).  Selection is
    argmax (greedy) or, with ``sampling`` (temperature > 0), a seeded device draw
    (top-k / top-p threshold + Gumbel-max, sampling.hip) — both inside the graph.
    ``greedy=False`` without ``sampling`` keeps the host-sampler mode: the graph
    stops after the penalty and the caller pushes the token.
    """

    def __init__(self, model: LlamaModel, repeat_penalty: float = 1.0, repeat_last_n: int = 128,
                 greedy: bool = True, use_graph: bool = True, steps_per_graph: int = 1,
                 sampling=None):
        if model.backend != "hip" or not model.all_local:
            raise ValueError("DeviceDecoder needs an all-local model on the hip backend")
        self.sampling = sampling if sampling is not None and not sampling.greedy else None
        if self.sampling is not None:
            greedy = True  # token chosen on the device: no host input between steps
        # device-selected decode needs no host input between steps, so several steps
        # can share one graph launch (fewer host round trips); host-sampled mode is 1
        self.k = max(1, int(steps_per_graph)) if greedy and use_graph else 1
        self.m = model
        self.penalty = float(repeat_penalty)
        self.last_n = int(repeat_last_n)
        self.greedy = greedy
        self.use_graph = use_graph
        self.bufs: DecodeBuffers = model.stack.decode_buffers(with_head=True)
        self.params: torch.Tensor | None = None  # device SampleParams (set_sampling)
        self.graph: torch.cuda.CUDAGraph | None = None
        # one graph per attention split cap (position buckets), see capture()
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.host_pos = 0  # device position of the next step (tracked on the host)
        self._layers = list(range(model.cfg.num_hidden_layers))
        # CAKE_FUSED_HEAD=0 keeps the four-launch tail (A/B)
        self._fuse_tail = os.environ.get("CAKE_FUSED_HEAD", "1") != "0"

    # the captured body
    def _step_body(self) -> None:
        from ...ops import hip as K
        b, m = self.bufs, self.m
        fused = self._fused_select()
        if not fused:
            K.embed(m.head.embed, b.tok, b.resid)
        m.stack.decode_step(b, self._layers, m.session)
        if fused:
            # greedy: lm_head + penalty + argmax + finalize + the next step's embedding
            # row in ONE launch (the step's input was embedded by the previous one, or
            # by _select_first)
            K.head_select(b.resid, m.head.norm, m.cfg.rms_norm_eps, m.head.lm_head, b.logits,
                          b.hist, b.hist_len, self.last_n if self.penalty != 1.0 else 0,
                          self.penalty, b.slot, b.sel_ticket, b.tok, b.pos, embed=m.head.embed)
            return
        K.norm_gemv_f32(b.resid, m.head.norm, m.cfg.rms_norm_eps, m.head.lm_head, b.logits)
        if self.penalty != 1.0:
            K.repeat_penalty(b.logits, b.hist, b.hist_len, self.last_n, self.penalty)
        if self.greedy:
            K.select_token(b.logits, b.slot, b.hist, b.hist_len, b.tok, b.pos, self.sampling,
                           b.thr, params=self.params)

    def _fused_select(self) -> bool:
        """Greedy argmax with no device parameter block: the fused head_select tail."""
        from ...ops import hip as K
        return (self.greedy and self.sampling is None and self.params is None
                and (self.penalty == 1.0 or self.last_n <= K.HEAD_SELECT_MAX_LAST_N)
                and self._fuse_tail)

    def set_sampling(self, sampling) -> None:
        """Per-request sampling configuration (None / temperature <= 0 = greedy).  The
        first call switches the selection to a device parameter block (one recapture);
        later calls only rewrite that block, so the captured graph is reused."""
        from ...ops import hip as K
        if self.params is None:
            self.params = torch.zeros(K.SAMPLE_PARAMS_WORDS, dtype=torch.int32,
                                      device=self.m.device)
            self.graph = None
            self.graphs = {}
            self.greedy = True
        self.sampling = sampling if sampling is not None and not sampling.greedy else None
        self.params.copy_(K.pack_sample_params(sampling))

    def profile_layers(self, reps: int = 3) -> list[float]:
        """Per-layer decode kernel time (ms): each layer's five launches
        captured as its own small graph and replayed between timing events, at the
        current device position (the K/V row it writes is the next step's, which that
        step rewrites).  Run between generations (--metrics)."""
        from ...ops import hip as K
        b, m = self.bufs, self.m
        if getattr(self, "_layer_graphs", None) is None:
            K.embed(m.head.embed, b.tok, b.resid)
            torch.cuda.synchronize()
            gs = []
            for li in self._layers:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    m.stack.decode_step(b, [li], m.session)
                gs.append(g)
            self._layer_graphs = gs
        K.embed(m.head.embed, b.tok, b.resid)
        out = [0.0] * len(self._layer_graphs)
        for _ in range(reps):
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(out) + 1)]
            evs[0].record()
            for i, g in enumerate(self._layer_graphs):
                g.replay()
                evs[i + 1].record()
            evs[-1].synchronize()
            for i in range(len(out)):
                out[i] += evs[i].elapsed_time(evs[i + 1]) / reps
        return out

    def capture(self) -> None:
        if not self.use_graph or self.graph is not None:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        # warm the kernels once outside capture on scratch state, then restore
        state = (self.bufs.tok, self.bufs.pos, self.bufs.hist_len, self.bufs.resid)
        saved = [t.clone() for t in state]
        hist = self.bufs.hist.clone()
        with torch.cuda.stream(s):
            self._step_body()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for t, v in zip(state, saved):
            t.copy_(v)
        self.bufs.hist.copy_(hist)
        self.bufs.slot.zero_()
        # Position buckets: the decode-attention grid is sized by its split cap, and
        # a max_seq-sized grid's idle workgroups cost every layer (8B, max_seq 4096:
        # 353 -> 368 tok/s at short context).  One graph per cap; launch() replays
        # the smallest whose cap covers the live length.
        from ...ops import hip as K
        self.graphs = {}
        for cap in K.attn_split_caps(self.m.stack.max_seq):
            g = torch.cuda.CUDAGraph()
            with K.attn_split_cap(cap), torch.cuda.graph(g):
                for _ in range(self.k):
                    self._step_body()
            self.graphs[cap] = g
        # bucket "1 split": attention and o_proj as one launch per layer (attn_oproj.hip),
        # for the live lengths whose attention is a single split
        st = self.m.stack
        if st.attn_oproj_ok() and not st.mk_enabled():
            g = torch.cuda.CUDAGraph()
            with K.attn_oproj_fused(), torch.cuda.graph(g):
                for _ in range(self.k):
                    self._step_body()
            self.graphs[1] = g
        self.graph = self.graphs[max(self.graphs)]
        torch.cuda.synchronize()

    def graph_set(self):
        """The bucket graphs as the native decode loop's GraphSet (built once)."""
        gs = getattr(self, "_graph_set", None)
        if gs is None or gs.graphs[-1] is not self.graphs[max(self.graphs)]:
            from ...ops import graph_loop as GL
            caps = sorted(self.graphs)
            index = {c: i for i, c in enumerate(caps)}
            by_graph = {id(self.graphs[c]): index[c] for c in caps}
            gs = self._graph_set = GL.GraphSet(
                [self.graphs[c] for c in caps], lambda t: by_graph[id(self._graph_for(t))],
                self.m.stack.max_seq)
        return gs

    def _graph_for(self, tk: int) -> torch.cuda.CUDAGraph:
        from ...ops import hip as K
        need = K.attn_splits(tk)
        for cap in sorted(self.graphs):
            if cap >= need:
                return self.graphs[cap]
        return self.graph

    def start(self, prompt: list[int]) -> int:
        """Prefill `prompt` at position 0 and select the first token (returned)."""
        m, b = self.m, self.bufs
        T = len(prompt)
        if T + 1 > m.stack.max_seq:
            raise ValueError("prompt longer than max_seq")
        m.stack.reset(m.session)
        h = m.embed(prompt)
        h = m.forward_hidden(h, 0)
        ids = torch.tensor(prompt, dtype=torch.int32)
        b.hist[:T].copy_(ids.to(m.device))
        b.hist_len.fill_(T)
        b.pos.fill_(T - 1)
        b.slot.zero_()
        m.head_logits(h[-1], out=b.logits)
        self.host_pos = T - 1
        return self._select_first()

    def _select_first(self) -> int:
        from ...ops import hip as K
        b = self.bufs
        if self.penalty != 1.0:
            K.repeat_penalty(b.logits, b.hist, b.hist_len, self.last_n, self.penalty)
        if self.greedy:
            K.select_token(b.logits, b.slot, b.hist, b.hist_len, b.tok, b.pos, self.sampling,
                           b.thr, params=self.params)
            if self._fused_select():  # the fused step body starts from the embedded token
                K.embed(self.m.head.embed, b.tok, b.resid)
            self.host_pos += 1
            return int(b.tok.item())
        raise RuntimeError("sampled mode: caller pushes the first token")

    def push(self, token: int) -> None:
        from ...ops import hip as K
        b = self.bufs
        src = torch.tensor([token], dtype=torch.int32, device=self.m.device)
        K.push_token(src, b.tok, b.hist, b.hist_len, b.pos)
        self.host_pos += 1

    def launch(self) -> None:
        """Enqueue `self.k` decode steps (one graph replay; async).  Raises instead of
        writing past the KV cache / token history (max_seq)."""
        if self.host_pos + self.k >= self.m.stack.max_seq:
            raise ValueError(f"decode step at position {self.host_pos} (+{self.k}) overruns "
                             f"max_seq {self.m.stack.max_seq}")
        if self.graph is not None:
            # live length of the last step of this replay (+1: sampled mode pushes)
            self._graph_for(self.host_pos + self.k + 1).replay()
        else:
            from ...ops import hip as K
            with K.attn_oproj_fused(K.attn_oproj_short(self.host_pos + self.k - 1)):
                self._step_body()
        if self.greedy:  # greedy steps advance pos on the device; sampled ones via push()
            self.host_pos += self.k

    def logits(self) -> torch.Tensor:
        return self.bufs.logits
