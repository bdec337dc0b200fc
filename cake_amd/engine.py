"""ctypes front of the native Llama engine (csrc/engine/llama_engine.cpp, libcake_engine.so).

The engine runs the whole text path of an all-local model in C++ — checkpoint load,
MFMA prefill, hipGraph-captured decode steps and the token loop — with no PyTorch in
the process's compute path.  This module only marshals arguments: the native CLI
(cake-cli, csrc/tools/cake_cli.cpp) calls the same C ABI directly, and the tests pin it
token-for-token to the Python DeviceDecoder (tests/test_engine_gpu.py).

Reference: cake-core/src/cake/master.rs:80-124 (generation loop) and
cake-core/src/models/llama3/llama.rs:72-138, 277-341 (the Llama generator).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from pathlib import Path
from typing import Callable

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libcake_engine.so"

TOKEN_CB = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32)


class EngineOpts(C.Structure):
    _fields_ = [("max_seq", C.c_int32), ("dtype", C.c_int32), ("device", C.c_int32),
                ("steps_per_graph", C.c_int32), ("init", C.c_int32), ("reserved", C.c_int32),
                ("seed", C.c_uint64)]


class PipeOpts(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("master_addr", C.c_char_p),
                ("hop_bf16", C.c_int32), ("hop_timeout_s", C.c_double),
                ("connect_timeout_s", C.c_double), ("owners", C.POINTER(C.c_int32)),
                ("n_owners", C.c_int32)]


class TPOpts(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("master_addr", C.c_char_p),
                ("timeout_s", C.c_double), ("connect_timeout_s", C.c_double)]


class RemoteOpts(C.Structure):
    _fields_ = [("worker_of", C.POINTER(C.c_int32)), ("n_layers", C.c_int32),
                ("workers", C.POINTER(C.c_char_p)), ("n_workers", C.c_int32),
                ("timeout_s", C.c_double)]


class EngineSampling(C.Structure):
    _fields_ = [("temperature", C.c_float), ("top_k", C.c_int32), ("top_p", C.c_float),
                ("seed", C.c_uint64), ("repeat_penalty", C.c_float),
                ("repeat_last_n", C.c_int32)]


class EngineStats(C.Structure):
    _fields_ = [("n_prompt", C.c_int32), ("n_generated", C.c_int32), ("prefill_s", C.c_double),
                ("decode_s", C.c_double), ("tokens_per_s", C.c_double), ("p50_ms", C.c_float),
                ("p99_ms", C.c_float)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} missing: run `python -m cake_amd.build`")
        L = C.CDLL(str(LIB_PATH))
        P, I = C.c_void_p, C.c_int32
        L.cake_engine_open.argtypes = [C.c_char_p, C.POINTER(EngineOpts), C.c_char_p, I]
        L.cake_engine_open.restype = P
        L.cake_engine_open_pp.argtypes = [C.c_char_p, C.POINTER(EngineOpts), C.POINTER(PipeOpts),
                                          C.c_char_p, I]
        L.cake_engine_open_pp.restype = P
        L.cake_engine_open_tp.argtypes = [C.c_char_p, C.POINTER(EngineOpts), C.POINTER(TPOpts),
                                          C.c_char_p, I]
        L.cake_engine_open_tp.restype = P
        L.cake_engine_open_remote.argtypes = [C.c_char_p, C.POINTER(EngineOpts),
                                              C.POINTER(RemoteOpts), C.c_char_p, I]
        L.cake_engine_open_remote.restype = P
        L.cake_engine_serve.argtypes = [P, C.c_char_p, I]
        L.cake_engine_serve.restype = I
        L.cake_engine_rank_info.argtypes = [P, C.POINTER(C.c_int32)]
        L.cake_engine_rank_info.restype = I
        L.cake_engine_info.argtypes = [P, C.POINTER(C.c_int32)]
        L.cake_engine_info.restype = I
        L.cake_engine_eos.argtypes = [P, C.POINTER(C.c_int32), I]
        L.cake_engine_eos.restype = I
        L.cake_engine_generate.argtypes = [P, C.POINTER(C.c_int32), I, I, C.POINTER(EngineSampling),
                                           C.POINTER(C.c_int32), I, TOKEN_CB, P,
                                           C.POINTER(C.c_int32), I, C.POINTER(EngineStats),
                                           C.c_char_p, I]
        L.cake_engine_generate.restype = I
        L.cake_engine_continue.argtypes = [P, I, C.POINTER(C.c_int32), I, TOKEN_CB, P,
                                           C.POINTER(C.c_int32), I, C.POINTER(EngineStats),
                                           C.c_char_p, I]
        L.cake_engine_continue.restype = I
        L.cake_engine_forced_logits.argtypes = [P, C.POINTER(C.c_int32), I, C.POINTER(C.c_int32),
                                                I, C.POINTER(C.c_float), C.c_char_p, I]
        L.cake_engine_forced_logits.restype = I
        L.cake_engine_walk.argtypes = [P, C.c_char_p, I]
        L.cake_engine_walk.restype = I
        L.cake_engine_prefill_logits.argtypes = [P, C.POINTER(C.c_int32), I,
                                                 C.POINTER(C.c_float), C.c_char_p, I]
        L.cake_engine_prefill_logits.restype = I
        L.cake_engine_close.argtypes = [P]
        L.cake_engine_close.restype = None
        _lib = L
    return _lib


@dataclass
class GenResult:
    tokens: list[int] = field(default_factory=list)
    n_prompt: int = 0
    prefill_s: float = 0.0
    decode_s: float = 0.0
    tokens_per_s: float = 0.0
    p50_ms: float = 0.0
    p99_ms: float = 0.0


class NativeLlama:
    """One model loaded by the native engine on one GPU."""

    def __init__(self, model_dir: str | Path, *, max_seq: int = 4096, dtype: str = "bf16",
                 device: int = 0, steps_per_graph: int = 1, rank: int = 0, world: int = 1,
                 master_addr: str = "127.0.0.1:29517", hop_bf16: bool = False,
                 hop_timeout_s: float = 30.0, connect_timeout_s: float = 600.0,
                 tp: bool = False, owners: list[int] | None = None, random_init: bool = False,
                 seed: int = 0, worker_of: list[int] | None = None,
                 workers: list[str] | None = None, remote_timeout_s: float = 120.0):
        """world > 1: one rank of a layer-sharded pipeline, or with tp=True of a tensor-
        parallel group (rank 0 generates; the others call :meth:`serve`).  Every rank of
        one group must be constructed concurrently.  ``owners`` (pipeline): the rank of
        every layer (:func:`owners_from_topology`); None = contiguous shards.
        ``random_init``: only ``config.json`` is read; the weights are seeded normal
        draws on the device (benchmarks of a named architecture, no checkpoint).
        ``workers`` / ``worker_of`` (single process): TCP workers ("host:port") and the
        worker index of every layer (-1 = local) — the master's Client
        (cake-core/src/cake/client.rs:23-133), contiguous runs batched per round trip."""
        if dtype not in ("bf16", "f16"):
            raise ValueError("native engine dtype: bf16 or f16")
        opts = EngineOpts(int(max_seq), 0 if dtype == "bf16" else 1, int(device),
                          max(1, int(steps_per_graph)), 1 if random_init else 0, 0,
                          int(seed) & 0xFFFFFFFFFFFFFFFF)
        err = C.create_string_buffer(1024)
        self._h = None
        if world > 1 and tp:
            self._addr = master_addr.encode()
            o = TPOpts(int(rank), int(world), self._addr, float(hop_timeout_s),
                       float(connect_timeout_s))
            self._h = lib().cake_engine_open_tp(str(model_dir).encode(), C.byref(opts),
                                                C.byref(o), err, len(err))
        elif world > 1:
            self._addr = master_addr.encode()
            own = None
            if owners is not None:
                own = (C.c_int32 * len(owners))(*[int(x) for x in owners])
            self._owners = own  # kept alive for the call
            pipe = PipeOpts(int(rank), int(world), self._addr, int(bool(hop_bf16)),
                            float(hop_timeout_s), float(connect_timeout_s),
                            C.cast(own, C.POINTER(C.c_int32)) if own is not None else None,
                            len(owners) if owners is not None else 0)
            self._h = lib().cake_engine_open_pp(str(model_dir).encode(), C.byref(opts),
                                                C.byref(pipe), err, len(err))
        elif workers:
            wo = (C.c_int32 * len(worker_of))(*[int(x) for x in worker_of])
            hs = (C.c_char_p * len(workers))(*[w.encode() for w in workers])
            self._remote = (wo, hs)  # kept alive for the call
            ro = RemoteOpts(C.cast(wo, C.POINTER(C.c_int32)), len(worker_of),
                            C.cast(hs, C.POINTER(C.c_char_p)), len(workers),
                            float(remote_timeout_s))
            self._h = lib().cake_engine_open_remote(str(model_dir).encode(), C.byref(opts),
                                                    C.byref(ro), err, len(err))
        else:
            self._h = lib().cake_engine_open(str(model_dir).encode(), C.byref(opts), err, len(err))
        if not self._h:
            raise RuntimeError(f"native engine: {err.value.decode(errors='replace')}")
        ri = (C.c_int32 * 4)()
        lib().cake_engine_rank_info(self._h, ri)
        self.rank, self.world, self.first_layer, self.end_layer = list(ri)
        info = (C.c_int32 * 8)()
        lib().cake_engine_info(self._h, info)
        (self.vocab_size, self.hidden_size, self.num_layers, self.num_heads, self.num_kv_heads,
         self.head_dim, self.intermediate_size, self.max_seq) = list(info)
        eos = (C.c_int32 * 16)()
        n = lib().cake_engine_eos(self._h, eos, 16)
        self.eos_ids = [int(eos[i]) for i in range(min(n, 16))]

    def walk(self) -> str:
        """The token's walk as "rank:first-last" layer runs (comma separated)."""
        buf = C.create_string_buffer(4096)
        lib().cake_engine_walk(self._h, buf, len(buf))
        return buf.value.decode()

    def serve(self) -> None:
        """Pipeline worker: run rank 0's prefill relays and replay announcements until it
        closes the pipeline."""
        err = C.create_string_buffer(1024)
        if lib().cake_engine_serve(self._h, err, len(err)):
            raise RuntimeError(f"native engine: {err.value.decode(errors='replace')}")

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().cake_engine_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def prefill_logits(self, prompt: list[int]):
        import numpy as np
        arr = (C.c_int32 * len(prompt))(*prompt)
        out = np.empty(self.vocab_size, dtype=np.float32)
        err = C.create_string_buffer(1024)
        rc = lib().cake_engine_prefill_logits(self._h, arr, len(prompt),
                                              out.ctypes.data_as(C.POINTER(C.c_float)), err,
                                              len(err))
        if rc:
            raise RuntimeError(f"native engine: {err.value.decode(errors='replace')}")
        return out

    def forced_logits(self, prompt: list[int], forced: list[int]):
        """Teacher forcing: f32 logits [len(forced) + 1, V] after the prompt and after each
        forced token (one eager decode step each, through every rank of the group)."""
        import numpy as np
        arr = (C.c_int32 * len(prompt))(*prompt)
        fa = (C.c_int32 * max(1, len(forced)))(*forced)
        out = np.empty((len(forced) + 1, self.vocab_size), dtype=np.float32)
        err = C.create_string_buffer(1024)
        rc = lib().cake_engine_forced_logits(self._h, arr, len(prompt), fa, len(forced),
                                             out.ctypes.data_as(C.POINTER(C.c_float)), err,
                                             len(err))
        if rc:
            raise RuntimeError(f"native engine: {err.value.decode(errors='replace')}")
        return out

    def generate(self, prompt: list[int], max_new: int, *, temperature: float = 0.0,
                 top_k: int | None = None, top_p: float | None = None, seed: int = 299792458,
                 repeat_penalty: float = 1.1, repeat_last_n: int = 128,
                 eos_ids: list[int] | None = None,
                 on_token: Callable[[int], bool | None] | None = None) -> GenResult:
        arr = (C.c_int32 * len(prompt))(*prompt)
        smp = EngineSampling(float(temperature or 0.0), int(top_k or 0), float(top_p or 0.0),
                             int(seed) & 0xFFFFFFFFFFFFFFFF, float(repeat_penalty),
                             int(repeat_last_n))
        return self._run(lambda eos_arr, n_eos, cb, out, stats, err: lib().cake_engine_generate(
            self._h, arr, len(prompt), int(max_new), C.byref(smp), eos_arr, n_eos, cb, None, out,
            max(1, max_new), stats, err, len(err)), max_new, eos_ids, on_token)

    def continue_(self, max_new: int, *, eos_ids: list[int] | None = None,
                  on_token: Callable[[int], bool | None] | None = None) -> GenResult:
        """Up to max_new more tokens after the last generate / continue (same sampling;
        the rate counts every token: all are decode steps)."""
        return self._run(lambda eos_arr, n_eos, cb, out, stats, err: lib().cake_engine_continue(
            self._h, int(max_new), eos_arr, n_eos, cb, None, out, max(1, max_new), stats, err,
            len(err)), max_new, eos_ids, on_token)

    def _run(self, call, max_new, eos_ids, on_token) -> GenResult:
        eos = list(eos_ids or [])
        eos_arr = (C.c_int32 * max(1, len(eos)))(*eos)
        out = (C.c_int32 * max(1, max_new))()
        stats = EngineStats()
        err = C.create_string_buffer(1024)
        errors: list[BaseException] = []

        def _tok(_ctx, t):
            try:
                return 1 if on_token(int(t)) else 0
            except BaseException as e:  # noqa: BLE001  (re-raised after the call)
                errors.append(e)
                return 1

        cb = TOKEN_CB(_tok) if on_token is not None else TOKEN_CB()
        rc = call(eos_arr, len(eos), cb, out, C.byref(stats), err)
        if errors:
            raise errors[0]
        if rc:
            raise RuntimeError(f"native engine: {err.value.decode(errors='replace')}")
        return GenResult([int(out[i]) for i in range(stats.n_generated)], stats.n_prompt,
                         stats.prefill_s, stats.decode_s, stats.tokens_per_s, stats.p50_ms,
                         stats.p99_ms)


def owners_from_topology(topology, num_layers: int, world: int) -> list[int]:
    """Layer -> pipeline rank of a topology: node i (file order) is rank i + 1, layers
    no node names stay on rank 0 (the master), as the reference's placement loop
    (cake-core/src/models/llama3/llama.rs:205-220, topology.rs:81-92)."""
    from .parallel.rccl_roles import owners_from_topology as f
    return f(topology, num_layers, world)


def remote_placement(topology, num_layers: int) -> tuple[list[int], list[str]]:
    """(worker_of, workers) of a topology for the master's TCP client: node i serves the
    layers it names (exact name lookup, topology.rs:81-92), the rest stay local."""
    nodes = list(topology.nodes)
    index = {id(n): i for i, n in enumerate(nodes)}
    worker_of = []
    for li in range(num_layers):
        node = topology.get_node_for_layer(f"model.layers.{li}")
        worker_of.append(-1 if node is None else index[id(node)])
    return worker_of, [n.host for n in nodes]


def write_config(path: str | Path, cfg) -> Path:
    """A model directory holding only ``config.json`` of ``cfg`` (random-init engines)."""
    import json
    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    (p / "config.json").write_text(json.dumps(cfg.to_hf_dict()))
    return p
