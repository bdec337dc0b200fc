"""Token sampling (candle-transformers ``LogitsProcessor`` semantics).

Reference: cake-core/src/models/llama3/llama.rs:34-48 picks
``Sampling::ArgMax`` when temperature <= 0, otherwise All / TopK / TopP /
TopKThenTopP with ``StdRng::seed_from_u64(seed)``.  We keep the selection
rules (softmax(logits / T); top-k keeps the k most probable; top-p walks the
probabilities in descending order zeroing everything after the running sum
reaches p; multinomial draw).  The RNG stream differs from Rust's StdRng
(ChaCha12), so sampled token ids are "parity unpinned"; the greedy path is
exact.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class SamplingConfig:
    temperature: float | None = 1.0
    top_k: int | None = None
    top_p: float | None = None
    repeat_penalty: float = 1.1
    repeat_last_n: int = 128
    seed: int = 299792458

    @property
    def greedy(self) -> bool:
        return self.temperature is None or self.temperature <= 0.0


class LogitsProcessor:
    def __init__(self, cfg: SamplingConfig, device="cpu"):
        self.cfg = cfg
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(cfg.seed)

    def sample(self, logits: torch.Tensor) -> int:
        logits = logits.float().reshape(-1)
        if self.cfg.greedy:
            return int(torch.argmax(logits).item())
        probs = torch.softmax(logits / float(self.cfg.temperature), dim=-1).cpu()
        k, p = self.cfg.top_k, self.cfg.top_p
        if k is not None and k > 0 and k < probs.numel():
            vals, idx = torch.topk(probs, k)
            mask = torch.zeros_like(probs)
            mask[idx] = 1.0
            probs = probs * mask
        if p is not None and 0.0 < p < 1.0:
            order = torch.argsort(probs, descending=True, stable=True)
            sp = probs[order]
            before = torch.cumsum(sp, 0) - sp  # running sum before each element
            sp = torch.where(before >= p, torch.zeros_like(sp), sp)
            probs = torch.zeros_like(probs).scatter_(0, order, sp)
        return int(torch.multinomial(probs, 1, generator=self.gen).item())
