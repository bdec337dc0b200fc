"""ctypes binding of ``libcake_kernels.so`` (the gfx950 HIP kernels).

The library exposes a plain C ABI; each entry point takes raw device pointers
plus the HIP stream to launch on.  We pass torch's *current* stream so that a
``torch.cuda.graph`` capture records our launches like any torch op.

On a machine with a GPU the library is mandatory: :func:`kernels` raises if it
is missing rather than silently falling back to PyTorch ops.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

_LIB_PATH = Path(__file__).resolve().parent.parent / "lib" / "libcake_kernels.so"
_lock = threading.Lock()
_lib = None

P = C.c_void_p
I = C.c_int
F = C.c_float
Z = C.c_size_t

# name -> argtypes (all return int hipError_t)
_SIGS = {
    "cake_attn_oproj": [I, P, P, P, P, I, I, I, I, F, P, I, I, P, I, P, P, P, P],
    "cake_attn_oproj_supported": [I, I, I, I],
    "cake_qkv_rope": [I, P, P, F, P, P, P, I, I, I, I, P, P, P, P, P, I, P],
    "cake_attn_set_prefetch": [I],
    "cake_swiglu": [I, P, P, F, P, P, I, I, P, P],
    "cake_gemv_x16": [I, P, P, I, I, P, I, P],
    "cake_gemv_norm_f32": [I, P, P, F, P, I, I, P, P],
    "cake_head_select": [I, P, P, F, P, I, I, P, P, P, I, F, P, P, P, P, I, P, P, P],
    "cake_attn_decode": [I, P, P, P, P, I, I, I, I, F, P, P, P, P],
    "cake_attn_set_impl": [I],
    "cake_attn_decode_heads": [I, P, P, P, P, I, I, I, I, F, P, P],
    "cake_attn_set_heads": [I, I],
    "cake_attn_set_head_prefetch": [I],
    "cake_attn_heads_max": [],
    "cake_attn_set_target_splits": [I],
    "cake_attn_set_single_max": [I],
    "cake_attn_set_min_keys": [I],
    "cake_attn_set_split_cap": [I],
    "cake_wave_reduce_probe": [P, P, P],
    "cake_embed": [I, P, P, I, I, P, P],
    "cake_rmsnorm": [I, P, P, F, I, I, P, P],
    "cake_rmsnorm_set_reg": [I],
    "cake_rope_kv": [I, P, P, P, I, I, I, I, I, I, P, I, I, P, P, P],
    "cake_silu_mul": [I, P, P, Z, P, P],
    "cake_silu_mul_rows": [I, P, Z, I, P, P],
    "cake_add_resid": [I, P, P, Z, P],
    "cake_repeat_penalty": [P, P, P, I, F, P],
    "cake_argmax": [P, I, P, P],
    "cake_finalize_token": [P, P, P, P, P, I, P],
    "cake_push_token": [P, P, P, P, P, I, P],
    "cake_gemv_set_tuning": [I, I, I, I],
    "cake_sample_threshold": [P, I, F, I, F, P, P],
    "cake_timestep_embed": [I, P, P, I, I, I, F, I, P, P],
    "cake_sched_step": [I, P, P, C.c_longlong, I, F, P, P, P, P, P],
    "cake_step_advance": [P, P],
    "cake_scale_copy": [I, P, C.c_longlong, F, I, P, P],
    "cake_to_rgb8": [I, P, I, I, I, I, P, P],
    "cake_attn512": [I, P, P, P, P, I, I, I, C.c_longlong, C.c_longlong, C.c_longlong,
                     C.c_longlong, C.c_longlong, C.c_longlong, C.c_longlong, C.c_longlong, F, P,
                     P],
    "cake_gumbel_argmax": [P, I, F, C.c_ulonglong, P, P, P, P],
    "cake_select_dev": [P, I, P, P, P, P, P],
    "cake_select_shard": [P, I, I, P, P, I, F, F, C.c_ulonglong, P, P],
    "cake_ar_sum": [P, P, I, I, P, P, P, P, I, I, C.c_double, P],
    "cake_ar_max_key": [P, P, P, P, P, I, I, C.c_double, P],
    "cake_ar_gather": [P, I, I, P, I, P, P, P, P, I, I, C.c_double, P],
}


class KernelError(RuntimeError):
    pass


def lib_path() -> Path:
    return Path(os.environ.get("CAKE_KERNEL_LIB", _LIB_PATH))


def kernels():
    """Load (once) and return the kernel library; raise if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            import torch  # noqa: F401  (HIP runtime must be loaded by torch first)

            path = lib_path()
            if not path.exists():
                raise KernelError(
                    f"{path} not built; run `python -m cake_amd.build` (hipcc gfx950)")
            lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
            for name, argtypes in _SIGS.items():
                if name in _OPTIONAL and not hasattr(lib, name):
                    continue  # csrc/experimental, built with CAKE_BUILD_EXPERIMENTAL=1
                fn = getattr(lib, name)
                fn.argtypes = argtypes
                fn.restype = _RESTYPE.get(name, C.c_int)
            _lib = lib
    return _lib


def available() -> bool:
    try:
        kernels()
        return True
    except (KernelError, OSError):
        return False


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise KernelError(f"{name} failed with hipError {rc}")

_SIGS.update({
    "cake_flash_attn": [I, P, P, P, P, I, I, I, I, I, I, P, F, I, I, P],
    "cake_flash_attn_ws": [I, P, P, P, P, I, I, I, I, I, I, P, F, I, I, P, C.c_longlong, P],
    "cake_flash_set_ksplit": [I],
    "cake_flash_set_impl": [I],
    "cake_flash_set_pair_min": [C.c_longlong],
    "cake_flash_set_nw": [I],
    "cake_groupnorm": [I, P, P, P, I, I, C.c_longlong, I, F, I, P, P, P],
    "cake_groupnorm_nhwc": [I, P, P, P, I, I, I, I, F, I, P, P, P, P, P],
    "cake_groupnorm_nhwc2": [I, P, P, I, P, P, P, I, I, I, I, F, I, P, P, P, P, P],
    "cake_groupnorm_nhwc_splits": [I],
    "cake_layernorm": [I, P, P, P, C.c_longlong, I, F, P, P],
    "cake_geglu": [I, P, C.c_longlong, I, P, P],
    "cake_stream_read": [P, Z, I, P, P],
    "cake_conv2d_nhwc": [I, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P],
    "cake_conv1x1_small": [I, P, P, P, P, I, I, I, I, I, P],
    "cake_conv2d_nhwc2": [I, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P],
})

_SIGS.update({
    "cake_mk_gstride": [I, I, I, I, I],
    "cake_mk_grid": [],
    "cake_mk_supported": [I, I, I, I, I],
    "cake_mk_decode": [I, P, I, I, I, I, I, I, I, F, F, P, P, P, P, P, C.c_double, P],
})
_RESTYPE = {"cake_mk_gstride": C.c_longlong, "cake_rmsnorm_set_reg": None}
# entry points of csrc/experimental (not in the default build)
_OPTIONAL = {"cake_mk_gstride", "cake_mk_grid", "cake_mk_supported", "cake_mk_decode",
             "cake_mk_set_stamps", "cake_mk_set_tuning",
             # fused decode attention + o_proj (measured slower: profiles/r5_attn_oproj_ab.md)
             "cake_attn_oproj", "cake_attn_oproj_supported", "cake_attn_oproj_ws_floats",
             "cake_attn_oproj_ticket_words"}
_SIGS["cake_mk_set_stamps"] = [P]
_SIGS["cake_mk_set_tuning"] = [I, I, I, I]
_SIGS["cake_attn_debug_drop_partials"] = [I]
