"""Master role (cake-core/src/cake/master.rs).

Loads the text or image generator for ``--model-type``; either serves the REST
API (``--api``) or runs ONE generation from the CLI flags: text streamed to
stdout, images written to ``images/image_{b}_{step}.png`` (the directory is
created — Appendix E Q15).  Text statistics use the reference formula:
tokens/s = (generated - 1) / time since the first token (master.rs:93-121,
guarded for a single token — Q13) plus p50/p99 per-token latency and TTFT.
"""
from __future__ import annotations

import logging
import sys
import time
from pathlib import Path
from typing import Callable

from .context import Context, hbm_mib, rss_mib
from .models.chat import Message

log = logging.getLogger("cake.master")


class Master:
    def __init__(self, ctx: Context, llm=None, sd=None):
        self.ctx = ctx
        self.llm = llm
        self.sd = sd
        self.last_stats: dict = {}
        if llm is None and sd is None:
            if ctx.model_type == "text-model":
                self.llm = _load_text(ctx)
            else:
                self.sd = _load_image(ctx)
        log.info("model loaded - mem=%.1f MiB", rss_mib())

    def run(self) -> None:
        a = self.ctx.args
        if getattr(a, "api", None):
            from .api.server import start
            start(self, a.api)
            return
        if self.llm is not None:
            self.llm.add_message(Message.system(a.system_prompt))
            self.llm.add_message(Message.user(a.prompt))

            def out(s: str) -> None:
                sys.stdout.write(s)
                sys.stdout.flush()
            self.generate_text(out)
            sys.stdout.write("\n")
        else:
            from .models.sd.args import ImageGenerationArgs
            Path("images").mkdir(exist_ok=True)
            step = [0]

            def save(images) -> None:
                for b, img in enumerate(images):
                    p = f"images/image_{b}_{step[0]}.png"
                    img.save(p)
                    log.info("saved %s", p)
                step[0] += 1
            self.generate_image(ImageGenerationArgs.from_cli(a), save)

    def reset(self) -> None:
        if self.llm is not None:
            self.llm.reset()

    def generate_text(self, stream: Callable[[str], None], max_tokens: int | None = None) -> dict:
        n = max_tokens if max_tokens is not None else self.ctx.args.sample_len
        llm = self.llm
        t_start = time.perf_counter()
        times: list[float] = []

        def on_token(tok) -> None:
            times.append(time.perf_counter())
            if not tok.is_end_of_stream:
                stream(str(tok))

        llm.stream(n, on_token)
        generated = llm.generated_tokens()
        stats = {"generated": generated}
        if times:
            stats["ttft_ms"] = (times[0] - t_start) * 1e3
        if len(times) > 1:
            dt = times[-1] - times[0]
            stats["tokens_per_sec"] = (len(times) - 1) / dt if dt > 0 else float("inf")
            lat = sorted((b - a) * 1e3 for a, b in zip(times, times[1:]))
            dev = getattr(llm, "last_stats", None)
            if dev is not None and dev.step_ms:  # device-timed steps when available
                lat = sorted(dev.step_ms)
            stats["p50_ms"] = lat[len(lat) // 2]
            stats["p99_ms"] = lat[min(len(lat) - 1, int(round(0.99 * (len(lat) - 1))))]
            native = getattr(llm, "latency_ms", None)  # the native engine's device timing
            pq = native() if callable(native) else None
            if pq is not None:
                stats["p50_ms"], stats["p99_ms"] = pq
        self._export(stats, t_start, times)
        log.info("%d tokens generated (%.2f token/s) p50=%.2fms p99=%.2fms ttft=%.1fms - mem=%.1f MiB",
                 generated, stats.get("tokens_per_sec", 0.0), stats.get("p50_ms", 0.0),
                 stats.get("p99_ms", 0.0), stats.get("ttft_ms", 0.0), rss_mib())
        self.last_stats = stats
        return stats

    def _export(self, stats: dict, t_start: float, times: list[float]) -> None:
        a = self.ctx.args
        if getattr(a, "metrics", None):
            import json
            extra = {}
            fn = getattr(self.llm, "metrics", None)
            if callable(fn):
                try:
                    extra = fn()
                except Exception as e:  # noqa: BLE001  (metrics never fail a generation)
                    log.warning("metrics: %s", e)
            with open(a.metrics, "a") as f:
                f.write(json.dumps({"ts": time.time(), "kind": "text", **stats,
                                    "rss_mib": round(rss_mib(), 1), **hbm_mib(),
                                    **extra}) + "\n")
        if getattr(a, "trace", None) and times:
            from .utils.trace import ChromeTrace
            tr = ChromeTrace()
            tr.t0 = t_start
            tr.add("prefill+first token", t_start, times[0])
            for i, (x, y) in enumerate(zip(times, times[1:])):
                tr.add(f"token {i + 1}", x, y)
            tr.save(a.trace)

    def generate_image(self, args, callback) -> None:
        self.sd.generate_image(args, callback)


def _load_text(ctx):
    """The native engine when it can serve this context (a GPU, 16-bit weights, graphs;
    topology workers through its TCP client), else the Python generator (CPU, f32,
    --no-graph, CAKE_NATIVE=0)."""
    from .models.llama3.native_generator import NativeLLM, native_eligible
    if native_eligible(ctx):
        topo = getattr(ctx, "topology", None)
        if topo is not None and getattr(topo, "nodes", None):
            log.info("text model on the native engine, TCP workers %s",
                     [f"{n.name}@{n.host}" for n in topo.nodes])
        else:
            log.info("text model on the native engine (libcake_engine.so)")
        return NativeLLM.load(ctx)
    from .models.llama3.generator import LLamaGenerator
    return LLamaGenerator.load(ctx)


def _load_image(ctx):
    """The native SD engine when every component is local on a GPU (csrc/engine/
    sd_engine.cpp), else the Python pipeline (also when the engine refuses the model,
    e.g. the tiny test architecture's 32-channel convolutions)."""
    from .models.sd.native_generator import NativeSDGenerator, native_sd_eligible
    from .models.sd.pipeline import SDGenerator
    if native_sd_eligible(ctx):
        try:
            gen = NativeSDGenerator.load(ctx)
            log.info("image generation on the native SD engine")
            return gen
        except Exception as e:  # noqa: BLE001  (the Python pipeline serves what it refuses)
            log.info("native SD engine unavailable (%s); using the Python pipeline", e)
    return SDGenerator.load(ctx)
