"""LLama text generator (cake-core/src/models/llama3/llama.rs:50-347).

``next_token(index)`` keeps the reference semantics exactly:
* first call: encode the chat history with the Llama-3 template, clear the KV
  cache, prefill all tokens at position 0 (llama.rs:140-166, 285-298);
* later calls: feed only the last token at ``index_pos`` (running count of
  fed tokens);
* repeat penalty over the last ``repeat_last_n`` tokens (prompt included) when
  ``repeat_penalty != 1`` (llama.rs:311-320); ArgMax when temperature <= 0,
  otherwise softmax sampling with top-k / top-p (llama.rs:34-48);
* ``Token.text`` = ``tokenizer.decode([id], skip_special=False)`` and
  ``is_end_of_stream`` when the id is an EOS id (config ``eos_token_id``
  scalar or list — Appendix E Q8 — else the ``</s>`` token).

Fast path: when every block is local on the HIP backend, the whole step
(layers + lm_head + penalty + argmax, or the seeded temperature / top-k /
top-p draw — the reference's default is temperature 1.0) is one hipGraph
replay (:class:`DeviceDecoder`) and :meth:`stream` overlaps the host token
read-back with the next step.  The device RNG is Philox keyed by the seed
(sampled ids are reproducible per seed but differ from Rust's StdRng stream:
"parity unpinned").
"""
from __future__ import annotations

from pathlib import Path
from typing import Callable

import torch

from ..base import TextGenerator, Token
from ..chat import History, Message
from ..sampling import LogitsProcessor, SamplingConfig
from ...ops import reference as R
from .model import DeviceDecoder, LlamaModel

DEFAULT_EOS_TOKEN = "</s>"


def load_tokenizer(model_dir: str | Path, eos_from_config: list[int]):
    from tokenizers import Tokenizer
    tok = Tokenizer.from_file(str(Path(model_dir) / "tokenizer.json"))
    eos = list(eos_from_config)
    if not eos:
        tid = tok.token_to_id(DEFAULT_EOS_TOKEN)
        if tid is not None:
            eos = [tid]
    return tok, set(eos)


class LLamaGenerator(TextGenerator):
    MODEL_NAME = "llama3"

    def __init__(self, model: LlamaModel, tokenizer, eos_ids: set[int],
                 sampling: SamplingConfig, use_graph: bool = True):
        self.model = model
        self.tokenizer = tokenizer
        self.eos_ids = set(eos_ids)
        self.sampling = sampling
        self.logits_processor = LogitsProcessor(sampling)
        self.history = History()
        self.tokens: list[int] = []
        self.generated = 0
        self.index_pos = 0
        self._dec: DeviceDecoder | None = None
        self._use_graph = use_graph
        self._per_request = False
        self.last_stats = None

    # ------------------------------------------------------------------ factory
    @classmethod
    def load(cls, ctx) -> "LLamaGenerator":
        from .factory import load_model
        from ...parallel.client import connect_remote_layers
        remote = connect_remote_layers(ctx)
        model = load_model(ctx.model_path, ctx.device, ctx.dtype, max_seq=ctx.max_seq_len,
                           remote=remote)
        tok, eos = load_tokenizer(ctx.model_path, model.cfg.eos_token_id)
        return cls(model, tok, eos, ctx.sampling, use_graph=not ctx.no_graph)

    # ------------------------------------------------------------------ TextGenerator
    def add_message(self, message: Message) -> None:
        self.history.append(message)

    def reset(self) -> None:
        self.tokens.clear()
        self.history.clear()
        self.model.reset()
        self.index_pos = 0
        self.generated = 0

    def generated_tokens(self) -> int:
        return self.generated

    def metrics(self) -> dict:
        """Extra fields for the --metrics sink: per-layer decode kernel ms (device path)."""
        if self._dec is None or not self._fast_path():
            return {}
        ms = self._dec.profile_layers()
        return {"layer_ms": [round(x, 4) for x in ms], "layers_ms_total": round(sum(ms), 3)}

    def set_sampling(self, sampling: SamplingConfig) -> None:
        """Sampling configuration of the next generation (API per-request temperature /
        top_k / top_p).  On the device path the decode graph reads it from device
        memory, so switching costs no recapture after the first switch."""
        self.sampling = sampling
        self.logits_processor = LogitsProcessor(sampling)
        self._per_request = True
        if self._dec is not None:
            self._dec.set_sampling(sampling)

    def _decode(self, tid: int) -> str | None:
        try:
            return self.tokenizer.decode([tid], skip_special_tokens=False)
        except Exception:  # noqa: BLE001  (reference logs and returns None)
            return None

    def _token(self, tid: int) -> Token:
        return Token(id=tid, text=self._decode(tid), is_end_of_stream=tid in self.eos_ids)

    def start_dialog_prompt(self) -> None:
        self.tokens = self.tokenizer.encode(self.history.encode_dialog_to_prompt(),
                                            add_special_tokens=False).ids
        self.model.reset()
        self.index_pos = 0

    def _fast_path(self) -> bool:
        return self.model.backend == "hip" and self.model.all_local

    def next_token(self, index: int) -> Token:
        if self.generated == 0:
            self.start_dialog_prompt()
        if self._fast_path():
            return self._next_token_device(index)
        if index > 0:
            ctx_tokens, ctx_index = self.tokens[-1:], self.index_pos
        else:
            ctx_tokens, ctx_index = list(self.tokens), 0
        logits = self.model.forward(ctx_tokens, ctx_index)
        if self.sampling.repeat_penalty != 1.0:
            start = max(0, len(self.tokens) - self.sampling.repeat_last_n)
            logits = R.apply_repeat_penalty(logits, self.sampling.repeat_penalty,
                                            self.tokens[start:])
        self.index_pos += len(ctx_tokens)
        tid = self.logits_processor.sample(logits)
        self.generated += 1
        self.tokens.append(tid)
        return self._token(tid)

    def _decoder(self) -> DeviceDecoder:
        if self._dec is None:
            self._dec = DeviceDecoder(self.model, repeat_penalty=self.sampling.repeat_penalty,
                                      repeat_last_n=self.sampling.repeat_last_n, greedy=True,
                                      use_graph=self._use_graph, sampling=self.sampling)
            if self._per_request:
                self._dec.set_sampling(self.sampling)
        return self._dec

    def _next_token_device(self, index: int) -> Token:
        dec = self._decoder()
        if index == 0 or self.generated == 0:
            tid = dec.start(self.tokens)
            dec.capture()
            self.index_pos = len(self.tokens)
        else:
            dec.launch()
            tid = int(dec.bufs.tok.item())
            self.index_pos += 1
        self.generated += 1
        self.tokens.append(tid)
        return self._token(tid)

    # ------------------------------------------------------------------ streaming
    def stream(self, max_tokens: int, on_token: Callable[[Token], None],
               stop_at_eos: bool = True) -> list[Token]:
        """Generate up to max_tokens tokens (first = prefill token), calling on_token."""
        out: list[Token] = []
        if max_tokens <= 0:
            return out
        first = self.next_token(0)
        out.append(first)
        on_token(first)
        if first.is_end_of_stream and stop_at_eos:
            return out
        # every further token needs a KV-cache row: clamp to the cache (max_seq)
        max_tokens = min(max_tokens, self.model.stack.max_seq - len(self.tokens) + 1)
        if not self._fast_path():
            for i in range(1, max_tokens):
                t = self.next_token(i)
                out.append(t)
                on_token(t)
                if t.is_end_of_stream and stop_at_eos:
                    break
            return out
        from .decode_loop import run_decode

        def cb(tid: int):
            t = self._token(tid)
            out.append(t)
            self.tokens.append(tid)
            self.generated += 1
            self.index_pos += 1
            on_token(t)

        self.last_stats = run_decode(self._decoder(), max_tokens - 1,
                                     self.eos_ids if stop_at_eos else None, cb)
        # the speculative step after EOS advanced the device state one token further
        torch.cuda.synchronize()
        return out
