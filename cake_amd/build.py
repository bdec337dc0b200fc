"""Native build driver: HIP kernels (gfx950) and the C++ host runtime.

Everything is compiled in-tree into ``cake_amd/lib/`` so the shared objects
travel with the repository snapshot to the GPU box:

* ``libcake_kernels.so`` — every ``csrc/kernels/*.hip`` file, ``hipcc
  --offload-arch=gfx950``; plain C ABI (``extern "C" cake_*``) driven from
  :mod:`cake_amd.ops.hip` through ctypes with torch's current HIP stream, so
  the launches are capturable in hipGraphs.  Also ``csrc/driver/*.cpp``: the
  native decode loop that replays the captured step graphs
  (:mod:`cake_amd.runtime.graph_loop`).
* ``libcake_runtime.so`` — ``csrc/runtime/*.cpp`` (topology parser, wire codec,
  safetensors mmap reader/writer, framed TCP transport), C ABI.
* ``cake-split-model`` — native executable (``csrc/tools/split_model.cpp``).
* ``cake-cli`` — the native entry point (``csrc/tools/cake_cli.cpp``): flags,
  validation and topology natively, compute runtime embedded in-process
  (libpython); ``libcake_runtime.so``'s ``cake_start_worker`` embeds the same way.

Object files are cached under ``build/`` keyed on mtimes of the source and the
shared headers, so re-running is cheap.

Usage: ``python -m cake_amd.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB = PKG / "lib"
BUILD = PKG.parent / "build" / "native"
ARCH = os.environ.get("CAKE_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CXX = shutil.which("g++") or "c++"

KERNEL_LIB = LIB / "libcake_kernels.so"
RUNTIME_LIB = LIB / "libcake_runtime.so"
SPLIT_TOOL = LIB / "cake-split-model"
CLI_TOOL = LIB / "cake-cli"


def _newer(src: Path, deps: list[Path], out: Path) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *deps] if p.exists())


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


# per-file hipcc flags: the GEMM's compile-time-unrolled interleaved schedule needs its
# lambdas fully inlined (below the default threshold the 128x128-per-wave tile keeps
# closures in scratch memory)
HIP_EXTRA = {"gemm": ["-mllvm", "-inline-threshold=100000"]}  # gemm.hip and gemm_inst_*.hip


def _compile_hip(src: Path, force: bool) -> Path:
    out = BUILD / "kernels" / (src.stem + ".o")
    out.parent.mkdir(parents=True, exist_ok=True)
    headers = sorted((CSRC / "kernels").glob("*.h"))
    if force or _newer(src, headers, out):
        _run([HIPCC, "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC",
              "-Wno-unused-result", "-munsafe-fp-atomics",
              *HIP_EXTRA.get(src.stem.split("_")[0], []),
              "-c", str(src), "-o", str(out)])
    return out


def _compile_cpp(src: Path, force: bool, extra: list[str] | None = None) -> Path:
    out = BUILD / "runtime" / (src.stem + ".o")
    out.parent.mkdir(parents=True, exist_ok=True)
    headers = sorted((CSRC / "runtime").glob("*.h")) + [CSRC / "engine" / "llama_engine.h"]
    if force or _newer(src, headers, out):
        _run([CXX, "-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
              "-fvisibility=hidden", *(extra or []), "-c", str(src), "-o", str(out)])
    return out


def _py_ext_flags() -> tuple[list[str], str]:
    import sysconfig

    import pybind11
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    return inc, sysconfig.get_config_var("EXT_SUFFIX") or ".so"


PY_EXT = LIB / "_cake_runtime"  # + EXT_SUFFIX

EXPERIMENTAL = os.environ.get("CAKE_BUILD_EXPERIMENTAL", "0") != "0"


def build_kernels(force: bool = False, jobs: int = 8) -> Path:
    # HIP kernels + the native graph-replay decode driver (host code on the HIP runtime).
    # csrc/experimental (the persistent decode engine, measured slower than the launch
    # path: profiles/r4_mk_summary.md) only with CAKE_BUILD_EXPERIMENTAL=1.
    srcs = sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "driver").glob("*.cpp"))
    if EXPERIMENTAL:
        srcs += sorted((CSRC / "experimental").glob("*.hip"))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile_hip(s, force), srcs))
    LIB.mkdir(parents=True, exist_ok=True)
    stale = [o for o in (BUILD / "kernels").glob("*.o") if o not in objs]
    for o in stale:  # an object of a source no longer built (experimental off) must go
        o.unlink()
    if force or stale or any(_newer(o, [], KERNEL_LIB) for o in objs):
        # hipBLASLt for the plain prefill GEMMs it measured faster on (driver/blaslt.cpp);
        # in a torch process the soname resolves to the copy torch already loaded
        # --no-undefined: a kernel whose host stub the compiler dropped fails here, not at
        # dlopen on the GPU box
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs),
              "-o", str(KERNEL_LIB), "-L/opt/rocm/lib", "-lhipblaslt", "-Wl,--no-undefined"])
    return KERNEL_LIB


def _embed_flags() -> tuple[list[str], list[str]]:
    """Compile / link flags to embed libpython (python3-config --embed equivalent)."""
    import sysconfig
    inc = [f"-I{sysconfig.get_paths()['include']}"]
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    libdir = sysconfig.get_config_var("LIBDIR") or "/usr/lib"
    return inc, [f"-L{libdir}", f"-lpython{ver}", "-ldl", "-lm", "-lpthread"]


def build_runtime(force: bool = False, jobs: int = 8) -> Path:
    """C++ host runtime: pybind11 module, C-ABI library, split-model tool and cake-cli."""
    rt = CSRC / "runtime"
    core_srcs = [rt / f"{n}.cpp" for n in ("json", "topology", "proto", "net", "safetensors",
                                            "server", "native_worker")]
    inc, ext = _py_ext_flags()
    einc, elink = _embed_flags()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        core = list(ex.map(lambda s: _compile_cpp(s, force), core_srcs))
        capi_f = ex.submit(_compile_cpp, rt / "capi.cpp", force)
        bind_f = ex.submit(_compile_cpp, rt / "bindings.cpp", force, inc)
        emb_f = ex.submit(_compile_cpp, rt / "embed.cpp", force, einc)
        capi, bind, emb = capi_f.result(), bind_f.result(), emb_f.result()
    LIB.mkdir(parents=True, exist_ok=True)
    pyext = PY_EXT.with_name(PY_EXT.name + ext)
    if force or any(_newer(o, [], pyext) for o in [*core, bind]):
        _run([CXX, "-shared", "-fPIC", *map(str, core), str(bind), "-o", str(pyext), "-lpthread",
              "-ldl"])
    if force or any(_newer(o, [], RUNTIME_LIB) for o in [*core, capi, emb]):
        _run([CXX, "-shared", "-fPIC", *map(str, core), str(capi), str(emb), "-o",
              str(RUNTIME_LIB), *elink])
    tool = CSRC / "tools" / "split_model.cpp"
    if force or _newer(tool, [*core, *sorted(rt.glob("*.h"))], SPLIT_TOOL):
        _run([CXX, "-O2", "-std=c++17", f"-I{rt}", str(tool), *map(str, core), "-o",
              str(SPLIT_TOOL), "-lpthread", "-ldl"])
    cli = CSRC / "tools" / "cake_cli.cpp"
    if force or _newer(cli, [*core, emb, *sorted(rt.glob("*.h")), CSRC / "engine" / "llama_engine.h"],
                       CLI_TOOL):
        _run([CXX, "-O2", "-std=c++17", f"-I{rt}", str(cli), *map(str, core), str(emb), "-o",
              str(CLI_TOOL), *elink])
    return pyext


ENGINE_LIB = LIB / "libcake_engine.so"


def build_engine(force: bool = False) -> Path:
    """Native engines (csrc/engine: Llama, Stable Diffusion): host C++ on the HIP runtime
    over the kernel library's C entry points, plus the runtime's JSON / safetensors
    readers."""
    rt = CSRC / "runtime"
    objs = [_compile_cpp(rt / f"{n}.cpp", force) for n in ("json", "safetensors", "net", "proto")]
    deps = [*sorted((CSRC / "engine").glob("*.h")), *sorted(rt.glob("*.h")),
            CSRC / "driver" / "graph_loop.h"]
    eng_objs = []
    for src in sorted((CSRC / "engine").glob("*.cpp")):  # llama_engine, sd_engine
        out = BUILD / "engine" / (src.stem + ".o")
        out.parent.mkdir(parents=True, exist_ok=True)
        if force or _newer(src, deps, out):
            _run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
                  "-Wno-unused-function", "-c", str(src), "-o", str(out)])
        eng_objs.append(out)
    if force or any(_newer(o, [], ENGINE_LIB) for o in [*eng_objs, *objs, KERNEL_LIB]):
        _run([HIPCC, "-shared", "-fPIC", *map(str, eng_objs), *map(str, objs), "-o",
              str(ENGINE_LIB), f"-L{LIB}", "-lcake_kernels", "-Wl,-rpath,$ORIGIN",
              "-Wl,--no-undefined"])
    return ENGINE_LIB


def build_all(force: bool = False, jobs: int = 8) -> None:
    build_kernels(force, jobs)
    build_engine(force)
    build_runtime(force, jobs)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--only", choices=["kernels", "engine", "runtime"], default=None)
    a = ap.parse_args(argv)
    if a.only in (None, "kernels"):
        print("built", build_kernels(a.force, a.jobs))
    if a.only in (None, "engine"):
        print("built", build_engine(a.force))
    if a.only in (None, "runtime"):
        print("built", build_runtime(a.force, a.jobs))
    return 0


if __name__ == "__main__":
    sys.exit(main())
