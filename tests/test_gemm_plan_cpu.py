"""GEMM tile plans on the CPU: the measured table (ops/gemm_tuned.json) and the three places
that name the tile configurations — the kernel table (csrc/kernels/gemm_kernel.h
CAKE_GEMM_CFGS), the Python planner (ops/gemm.py CFG_TILES) and the native engine's planner
(csrc/engine/engine_util.h, shared by the Llama and SD engines) — must agree, or a tuned plan launches a tile the library
does not have."""
import json
import re
from pathlib import Path

from cake_amd.ops import gemm as G

ROOT = Path(__file__).resolve().parents[1]


def _kernel_cfgs() -> dict:
    src = (ROOT / "cake_amd/csrc/kernels/gemm_kernel.h").read_text()
    body = src[src.index("#define CAKE_GEMM_CFGS(X)"):]
    body = body[:body.index("\n\n")]
    cfgs = {int(m[0]): (int(m[1]), int(m[2]), int(m[3]), int(m[4]))
            for m in re.findall(r"X\((\d+),\s*(\d+),\s*(\d+),\s*(\d+),\s*(\d+),", body)}
    # the two 256x256 kernels of their own: ping-pong (8 waves, 2 x 4) and register-staged
    # (4 waves, 2 x 2)
    for hdr, name, waves in (("gemm_pp.h", "kPPCfg", (2, 4)), ("gemm_rs.h", "kRSCfg", (2, 2)),
                             ("gemm_4w.h", "k4WCfg", (2, 2)), ("gemm_4w.h", "k4WCfg192", (2, 2)),
                             ("gemm_4w.h", "k4WCfg128", (2, 2))):
        t = (ROOT / "cake_amd/csrc/kernels" / hdr).read_text()
        cid = int(re.search(name + r" = (\d+);", t).group(1))
        tile = {"k4WCfg192": (256, 192), "k4WCfg128": (128, 256)}.get(name, (256, 256))
        cfgs[cid] = tile + waves
    # the three-barrier twins of the four-wave tiles: cfg + k4WSched, same tile
    t = (ROOT / "cake_amd/csrc/kernels/gemm_4w.h").read_text()
    sched = int(re.search(r"k4WSched = (\d+);", t).group(1))
    for name in ("k4WCfg", "k4WCfg192", "k4WCfg128"):
        cid = int(re.search(name + r" = (\d+);", t).group(1))
        cfgs[cid + sched] = cfgs[cid]
    return cfgs


def test_tile_tables_agree():
    kern = _kernel_cfgs()
    assert set(kern) == set(G.CFG_TILES)
    for cfg, (bm, bn, wm, wn) in kern.items():
        assert G.CFG_TILES[cfg] == (bm, bn), cfg
        # the gated epilogues need 32-column wave tiles; the others are refused up front
        assert ((bn // wn) % 32 == 0) == (cfg not in G.NO_GATED), cfg
    eng = (ROOT / "cake_amd/csrc/engine/engine_util.h").read_text()
    known = re.search(r"static const int known\[\] = \{([^}]*)\}", eng).group(1)
    assert {int(x) for x in known.replace("\n", " ").split(",")} == set(G.CFG_TILES)
    assert set(G._SLOTS) == set(G.CFG_TILES) and set(G._EFF) == set(G.CFG_TILES)


def test_tuned_table_entries_are_launchable():
    table = json.loads((ROOT / "cake_amd/ops/gemm_tuned.json").read_text())["entries"]
    assert table
    seen = set()
    for e in table:
        # one MFMA plan per shape, and at most one library (A/B arm) entry beside it
        key = (e["M"], e["Nv"], e["K"], e["epi"], e["cfg"] == G.LIB)
        assert key not in seen, f"duplicate plan {key}"
        seen.add(key)
        assert e["splits"] >= 1 and e["epi"] in G.EPI, e
        if e["cfg"] == G.LIB:  # the library GEMM: only the epilogues it carries
            assert e["epi"] in G.LIB_EPIS and e["splits"] == 1, e
            continue
        assert e["cfg"] in G.CFG_TILES, e
        if e["epi"] in ("swiglu", "geglu"):
            assert e["cfg"] not in G.NO_GATED and e["Nv"] % 32 == 0, e
        assert e["K"] % 8 == 0, e
        if e["cfg"] in G.K64_ONLY:
            assert e["K"] % 64 == 0 and (e["K"] // e["splits"]) % 64 == 0, e


def test_plan_uses_measured_entries():
    table = json.loads((ROOT / "cake_amd/ops/gemm_tuned.json").read_text())["entries"]
    # (entries naming the library GEMM are read only under CAKE_GEMM_LIB=1)
    e = next(x for x in table if x["M"] >= 512 and x["cfg"] != G.LIB)
    assert G.plan(e["M"], e["Nv"], e["K"], e["epi"]) == (e["cfg"], e["splits"])
    # a nearby M (within 2x) reuses the measured tile without split-K
    cfg, splits = G.plan(e["M"] + 8, e["Nv"], e["K"], e["epi"])
    assert (cfg in G.CFG_TILES or cfg == G.LIB) and splits == 1
    # an unmeasured shape falls back to the cost model
    cfg, splits = G.plan(333, 4448, 1024, "store")
    assert cfg in G.CFG_TILES and splits >= 1


def test_library_gemm_is_off_the_default_path(monkeypatch):
    """No default plan names the library GEMM (hipBLASLt): every prefill projection runs an
    MFMA kernel.  The measured library entries (profiles/r5_gemm_lib.jsonl) stay in the
    table as the A/B arm, read only under CAKE_GEMM_LIB=1 — by both planners, for the same
    epilogues."""
    eng = (ROOT / "cake_amd/csrc/engine/engine_util.h").read_text()
    assert re.search(r"constexpr int kGemmLib = (-?\d+);", eng).group(1) == str(G.LIB)
    body = eng[eng.index("const bool lib = "):]
    body = body[:body.index(";")]
    assert "lib_ok &&" in body and 'getenv("CAKE_GEMM_LIB")' in eng
    assert set(re.findall(r'ep == "(\w+)"', body)) == set(G.LIB_EPIS)
    monkeypatch.setattr(G, "_plans", {})
    assert all(e["cfg"] != G.LIB for e in G._TUNED)
    assert G.plan(2048, 28672, 4096, "swiglu")[0] in G.CFG_TILES   # 8B gate|up, 2048 tokens
    assert G.plan(2048, 6144, 4096, "store")[0] in G.CFG_TILES     # 8B q|k|v
    assert G.plan(2048, 1280, 5120, "add16")[0] in G.CFG_TILES     # SD shapes
    monkeypatch.setenv("CAKE_GEMM_LIB", "1")
    lib_table = G._load_tuned()
    assert any(e["cfg"] == G.LIB for e in lib_table)
    monkeypatch.setattr(G, "_TUNED", lib_table)
    monkeypatch.setattr(G, "_plans", {})
    assert G.plan(2048, 28672, 4096, "swiglu")[0] == G.LIB


def test_nearest_measured_plan_scales_split_k(monkeypatch):
    """A shape measured at M with split-K s, asked at M' within 2x: the same tile with
    s * M / M' splits (a power of two >= 1) — the grid fill the split was chosen for —
    and a library entry stays a library plan; the engine planner applies the same rule."""
    monkeypatch.setattr(G, "_TUNED", [
        {"M": 32, "Nv": 4096, "K": 14336, "epi": "resid32", "cfg": 13, "splits": 4},
        {"M": 1024, "Nv": 4096, "K": 14336, "epi": "resid32", "cfg": G.LIB, "splits": 1}])
    monkeypatch.setattr(G, "_plans", {})
    assert G.plan(32, 4096, 14336, "resid32") == (13, 4)
    assert G.plan(64, 4096, 14336, "resid32") == (13, 2)
    assert G.plan(40, 4096, 14336, "resid32") == (13, 2)
    assert G.plan(20, 4096, 14336, "resid32") == (13, 4)   # 6.4 -> 4
    assert G.plan(1500, 4096, 14336, "resid32") == (G.LIB, 1)
    assert G.plan_mfma(1500, 4096, 14336, "resid32")[0] in G.CFG_TILES
    eng = (ROOT / "cake_amd/csrc/engine/engine_util.h").read_text()
    assert "near->splits * near->M / std::max(M, 1LL)" in eng


def test_kernel_library_exports_the_library_gemm():
    """libcake_kernels.so carries the hipBLASLt entry point the plans name (and resolves
    its hipBLASLt dependency: the load itself needs no GPU)."""
    import ctypes

    import pytest

    import torch  # noqa: F401  (the HIP runtime as the package loads it)
    from cake_amd.ops import _lib
    path = _lib.lib_path()
    if not path.exists():
        pytest.skip("kernel library not built")
    lib = ctypes.CDLL(str(path))
    assert hasattr(lib, "cake_blaslt_gemm") and hasattr(lib, "cake_gemm")
    assert hasattr(lib, "cake_rmsnorm_set_reg")
