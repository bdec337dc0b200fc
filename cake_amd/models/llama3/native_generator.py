"""LLama text generator on the native engine (libcake_engine.so).

The reference's generator (cake-core/src/models/llama3/llama.rs:50-347) behind the
TextGenerator contract, with the whole token loop in C++: the chat template and the
tokenizer stay here (Python ``tokenizers``, the HF Rust library the reference links),
prefill, the graph-replayed decode, the repeat penalty and the sampling run in the
engine.  One class covers every native mode — all-local on one GPU, a pipeline rank 0
(the topology's placement, device hops) and a tensor-parallel rank 0 — so the REST API
(api/server.py, ``--api``) and the CLI master serve from the same engine the bench
measures.

Sampling: greedy, or the seeded temperature / top-k / top-p draw of the engine (device
Gumbel-max keyed by (seed, step): reproducible per seed, "parity unpinned" against the
reference's StdRng stream, as in the Python device path).
"""
from __future__ import annotations

from typing import Callable

from ..base import TextGenerator, Token
from ..chat import History, Message
from ..sampling import SamplingConfig


class NativeLLM(TextGenerator):
    MODEL_NAME = "llama3"

    def __init__(self, engine, tokenizer, eos_ids, sampling: SamplingConfig):
        self.eng = engine
        self.tokenizer = tokenizer
        self.eos_ids = set(eos_ids)
        self.sampling = sampling
        self.history = History()
        self.tokens: list[int] = []
        self.generated = 0
        self.last_stats = None
        self.last_result = None

    # ------------------------------------------------------------------ factory
    @classmethod
    def load(cls, ctx, engine=None) -> "NativeLLM":
        """All-local engine on ctx.device (or rank 0's ``engine`` of a running group)."""
        from .generator import load_tokenizer
        from ...engine import NativeLlama
        if engine is None:
            kw = {}
            topo = getattr(ctx, "topology", None)
            if topo is not None and getattr(topo, "nodes", None):
                from ...engine import remote_placement
                from .config import LlamaConfig
                L = LlamaConfig.from_path(ctx.model_path).num_hidden_layers
                worker_of, workers = remote_placement(topo, L)
                if any(w >= 0 for w in worker_of):
                    kw = dict(worker_of=worker_of, workers=workers)
            engine = NativeLlama(ctx.model_path, max_seq=ctx.max_seq_len,
                                 dtype=_dtype_name(ctx.dtype), device=ctx.device.index or 0, **kw)
        tok, eos = load_tokenizer(ctx.model_path, engine.eos_ids)
        return cls(engine, tok, eos, ctx.sampling)

    # ------------------------------------------------------------------ TextGenerator
    def add_message(self, message: Message) -> None:
        self.history.append(message)

    def reset(self) -> None:
        self.history.clear()
        self.tokens.clear()
        self.generated = 0

    def generated_tokens(self) -> int:
        return self.generated

    def set_sampling(self, sampling: SamplingConfig) -> None:
        """Per-request sampling (API): every generate call carries it to the engine."""
        self.sampling = sampling

    def latency_ms(self) -> tuple[float, float] | None:
        """(p50, p99) device time per decode token of the last generation."""
        r = self.last_result
        if r is None or not r.p50_ms:
            return None
        return float(r.p50_ms), float(r.p99_ms)

    def metrics(self) -> dict:
        r = self.last_result
        if r is None:
            return {}
        return {"engine": "native", "prefill_ms": round(r.prefill_s * 1e3, 3),
                "engine_tokens_per_s": round(r.tokens_per_s, 3),
                **({"walk": self.eng.walk()} if self.eng.world > 1 else {})}

    def _token(self, tid: int) -> Token:
        try:
            text = self.tokenizer.decode([tid], skip_special_tokens=False)
        except Exception:  # noqa: BLE001  (reference logs and returns None)
            text = None
        return Token(id=tid, text=text, is_end_of_stream=tid in self.eos_ids)

    def _kw(self) -> dict:
        s = self.sampling
        return dict(temperature=0.0 if s.greedy else float(s.temperature),
                    top_k=s.top_k, top_p=s.top_p, seed=int(s.seed),
                    repeat_penalty=float(s.repeat_penalty), repeat_last_n=int(s.repeat_last_n))

    def _prompt(self) -> list[int]:
        return self.tokenizer.encode(self.history.encode_dialog_to_prompt(),
                                     add_special_tokens=False).ids

    def next_token(self, index: int) -> Token:
        """The reference's per-token call: the first prefills the chat prompt, every
        later one is one more decode step of the same generation."""
        if self.generated == 0:
            self.tokens = self._prompt()
            r = self.eng.generate(self.tokens, 1, eos_ids=[], **self._kw())
        else:
            r = self.eng.continue_(1, eos_ids=[])
        tid = r.tokens[0]
        self.tokens.append(tid)
        self.generated += 1
        return self._token(tid)

    def stream(self, max_tokens: int, on_token: Callable[[Token], None],
               stop_at_eos: bool = True) -> list[Token]:
        """Up to max_tokens tokens (the first from the prefill), streamed as they are read
        back; stops after an EOS id (inclusive) unless stop_at_eos is False."""
        out: list[Token] = []
        if max_tokens <= 0:
            return out
        self.tokens = self._prompt()
        room = self.eng.max_seq - len(self.tokens) - 3
        if room <= 0:
            raise RuntimeError("prompt does not fit the KV cache (--max-seq-len)")

        def cb(tid: int) -> None:
            t = self._token(tid)
            out.append(t)
            self.tokens.append(tid)
            self.generated += 1
            on_token(t)
        self.last_result = self.eng.generate(
            self.tokens, min(max_tokens, room), eos_ids=sorted(self.eos_ids) if stop_at_eos else [],
            on_token=cb, **self._kw())
        return out


def _dtype_name(dtype) -> str:
    import torch
    if dtype == torch.bfloat16:
        return "bf16"
    if dtype == torch.float16:
        return "f16"
    raise ValueError(f"native engine dtype: bf16 or f16, not {dtype}")


def native_eligible(ctx, remote: bool = False) -> bool:
    """The native engine serves this context: a GPU, a 16-bit dtype, graphs on, and
    CAKE_NATIVE != 0 (``remote`` = a placement it cannot serve)."""
    import os

    import torch
    if os.environ.get("CAKE_NATIVE", "1") == "0" or remote:
        return False
    if ctx.device.type != "cuda" or getattr(ctx, "no_graph", False):
        return False
    if ctx.dtype not in (torch.float16, torch.bfloat16):
        return False
    from ...engine import LIB_PATH
    return LIB_PATH.exists()
