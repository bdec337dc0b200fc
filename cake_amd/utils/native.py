"""Loader for the native host runtime module (``cake_amd/lib/_cake_runtime*.so``)."""
from __future__ import annotations

import importlib.machinery
import importlib.util
import sysconfig
from pathlib import Path

_LIB = Path(__file__).resolve().parent.parent / "lib"
_mod = None


def runtime():
    """Return the `_cake_runtime` pybind11 module (built by `python -m cake_amd.build`)."""
    global _mod
    if _mod is None:
        path = _LIB / ("_cake_runtime" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
        if not path.exists():
            raise ImportError(f"{path} missing: run `python -m cake_amd.build --only runtime`")
        loader = importlib.machinery.ExtensionFileLoader("_cake_runtime", str(path))
        spec = importlib.util.spec_from_file_location("_cake_runtime", path, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _mod = mod
    return _mod
