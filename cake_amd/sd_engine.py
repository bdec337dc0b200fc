"""ctypes front of the native Stable Diffusion engine (csrc/engine/sd_engine.cpp, in
libcake_engine.so).

The engine runs a whole image generation in C++ — both text encoders, the guided
denoising loop (one hipGraph replay per step after the first) and the VAE decode — over
the same gfx950 kernels, in the same order, as the Python pipeline
(models/sd/pipeline.py), which the tests pin it against component by component and
image by image (tests/test_sd_engine_gpu.py).  Tokenization stays here (HF
``tokenizers``); the engine takes padded CLIP ids.

Reference: cake-core/src/models/sd/sd.rs:320-532 (generate_image), unet.rs, vae.rs, clip.rs.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from .engine import LIB_PATH, lib as _engine_lib

N_TOK = 77


class SdOpts(C.Structure):
    _fields_ = [("version", C.c_char_p), ("width", C.c_int32), ("height", C.c_int32),
                ("dtype", C.c_int32), ("device", C.c_int32), ("init", C.c_int32),
                ("autotune", C.c_int32), ("tiny", C.c_int32), ("seed", C.c_uint64),
                ("unet_path", C.c_char_p), ("vae_path", C.c_char_p), ("clip_path", C.c_char_p),
                ("clip2_path", C.c_char_p), ("parts", C.c_int32),
                ("remote_unet", C.c_char_p), ("remote_vae", C.c_char_p),
                ("remote_clip", C.c_char_p), ("remote_clip2", C.c_char_p),
                ("remote_timeout_s", C.c_double)]


PARTS = {"unet": 1, "vae": 2, "clip": 4, "clip2": 8}


class SdSplitOpts(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("master_addr", C.c_char_p),
                ("timeout_s", C.c_double), ("connect_timeout_s", C.c_double),
                ("owners", C.POINTER(C.c_int32)), ("n_owners", C.c_int32)]


class SdGenArgs(C.Structure):
    _fields_ = [("cond", C.POINTER(C.c_int32)), ("uncond", C.POINTER(C.c_int32)),
                ("cond2", C.POINTER(C.c_int32)), ("uncond2", C.POINTER(C.c_int32)),
                ("n_steps", C.c_int32), ("guidance", C.c_float), ("seed", C.c_uint64),
                ("init_noise", C.POINTER(C.c_float)), ("use_graph", C.c_int32),
                ("t_start", C.c_int32), ("init_latents", C.POINTER(C.c_float)),
                ("bsize", C.c_int32), ("intermediary", C.c_int32),
                ("on_image", C.c_void_p), ("cb_ctx", C.c_void_p)]


# on_image(cb_ctx, step, n_images, rgb [n_images, H, W, 3])
IMAGE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_uint8))


class SdResult(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("n_steps", C.c_int32),
                ("text_s", C.c_double), ("denoise_s", C.c_double), ("vae_s", C.c_double)]


_bound = False


def lib() -> C.CDLL:
    global _bound
    L = _engine_lib()
    if not _bound:
        P, I, F = C.c_void_p, C.c_int32, C.c_float
        FP = C.POINTER(C.c_float)
        L.cake_sd_open.argtypes = [C.c_char_p, C.POINTER(SdOpts), C.c_char_p, I]
        L.cake_sd_open.restype = P
        L.cake_sd_generate.argtypes = [P, C.POINTER(SdGenArgs), C.POINTER(C.c_uint8), FP,
                                       C.POINTER(C.c_double), C.POINTER(SdResult), C.c_char_p, I]
        L.cake_sd_generate.restype = I
        L.cake_sd_close.argtypes = [P]
        L.cake_sd_close.restype = None
        L.cake_sd_info.argtypes = [P, C.POINTER(C.c_int32)]
        L.cake_sd_info.restype = None
        L.cake_sd_text.argtypes = [P, I, C.POINTER(C.c_int32), I, FP, C.c_char_p, I]
        L.cake_sd_text.restype = I
        L.cake_sd_unet.argtypes = [P, FP, I, F, FP, FP, C.c_char_p, I]
        L.cake_sd_unet.restype = I
        L.cake_sd_vae_decode.argtypes = [P, FP, FP, C.c_char_p, I]
        L.cake_sd_vae_decode.restype = I
        L.cake_sd_vae_encode.argtypes = [P, FP, FP, C.c_char_p, I]
        L.cake_sd_vae_encode.restype = I
        L.cake_sd_vae_encode_remote.argtypes = [P, FP, FP, C.c_char_p, I]
        L.cake_sd_vae_encode_remote.restype = I
        L.cake_sd_open_split.argtypes = [C.c_char_p, C.POINTER(SdOpts), C.POINTER(SdSplitOpts),
                                         C.c_char_p, I]
        L.cake_sd_open_split.restype = P
        L.cake_sd_serve.argtypes = [P, C.c_char_p, I]
        L.cake_sd_serve.restype = I
        L.cake_sd_split_info.argtypes = [P, C.POINTER(C.c_int32)]
        L.cake_sd_split_info.restype = None
        _bound = True
    return L


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _ids(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _ip(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_int32))


@dataclass
class SdImage:
    rgb: np.ndarray                      # [H, W, 3] u8 ([bsize, H, W, 3] when bsize > 1)
    latents: np.ndarray                  # [4, H/8, W/8] f32 (final, before the VAE; batched
                                         # likewise)
    step_s: list[float] = field(default_factory=list)
    text_s: float = 0.0
    denoise_s: float = 0.0
    vae_s: float = 0.0


class NativeSD:
    """One Stable Diffusion model on one GPU, every component local."""

    def __init__(self, model_dir: str, version: str | None = None, width: int = 0,
                 height: int = 0, dtype: str = "f16", device: int = 0,
                 random_init: bool = False, seed: int = 0, autotune: bool = True,
                 paths: dict | None = None, parts=None, remote: dict | None = None,
                 remote_timeout_s: float = 120.0, rank: int = 0, world: int = 1,
                 master_addr: str = "127.0.0.1:29533", hop_timeout_s: float = 60.0,
                 connect_timeout_s: float = 600.0, owners: list[int] | None = None):
        """remote: component -> "host:port" of the TCP worker serving it (the topology's
        unet / vae / clip / clip2); those are not loaded here.  world > 1: one rank of a
        split UNet over one process per GPU (sd_engine.h CakeSdSplitOpts): rank 0
        generates, the others call :meth:`serve`; every rank of the group must be
        constructed concurrently."""
        if dtype not in ("f16", "bf16"):
            raise ValueError("native SD engine dtype: f16 or bf16")
        p = paths or {}
        rm = remote or {}
        self.remote = dict(rm)
        self._keep = [x.encode() if x else None for x in
                      (version, p.get("unet"), p.get("vae"), p.get("clip"), p.get("clip2"),
                       rm.get("unet"), rm.get("vae"), rm.get("clip"), rm.get("clip2"))]
        o = SdOpts(version=self._keep[0], width=int(width), height=int(height),
                   dtype=0 if dtype == "bf16" else 1, device=int(device),
                   init=1 if random_init else 0, autotune=1 if autotune else 0, tiny=0,
                   seed=int(seed), unet_path=self._keep[1], vae_path=self._keep[2],
                   clip_path=self._keep[3], clip2_path=self._keep[4],
                   parts=0 if parts is None else sum(PARTS[p] for p in parts),
                   remote_unet=self._keep[5], remote_vae=self._keep[6],
                   remote_clip=self._keep[7], remote_clip2=self._keep[8],
                   remote_timeout_s=float(remote_timeout_s))
        err = C.create_string_buffer(1024)
        if world > 1:
            own = None
            if owners is not None:
                own = (C.c_int32 * len(owners))(*[int(x) for x in owners])
            self._split_keep = (own, master_addr.encode())
            sp = SdSplitOpts(int(rank), int(world), self._split_keep[1], float(hop_timeout_s),
                             float(connect_timeout_s),
                             C.cast(own, C.POINTER(C.c_int32)) if own is not None else None,
                             len(owners) if owners is not None else 0)
            self._h = lib().cake_sd_open_split(str(model_dir).encode(), C.byref(o), C.byref(sp),
                                               err, 1024)
        else:
            self._h = lib().cake_sd_open(str(model_dir).encode(), C.byref(o), err, 1024)
        if not self._h:
            raise RuntimeError(f"native SD engine: {err.value.decode(errors='replace')}")
        info = (C.c_int32 * 6)()
        lib().cake_sd_info(self._h, info)
        self.width, self.height, self.context_dim, self._dt, d1, d2 = (int(x) for x in info)
        self.text_dims = (d1, d2)

    def split_info(self) -> dict:
        """rank, world, UNet stages, ranks used, and this rank's stage range."""
        o = (C.c_int32 * 6)()
        lib().cake_sd_split_info(self._h, o)
        return dict(zip(("rank", "world", "stages", "ranks_used", "first", "end"),
                        (int(x) for x in o)))

    def serve(self) -> None:
        """Split-UNet ranks > 0: run rank 0's generations until it closes the group."""
        err = C.create_string_buffer(1024)
        self._check(lib().cake_sd_serve(self._h, err, 1024), err)

    def _check(self, rc: int, err) -> None:
        if rc != 0:
            raise RuntimeError(f"native SD engine: {err.value.decode(errors='replace')}")

    def generate(self, cond, uncond=None, cond2=None, uncond2=None, n_steps: int = 30,
                 guidance: float = 7.5, seed: int = 0, init_noise=None,
                 use_graph: bool = True, init_latents=None, t_start: int = 0,
                 bsize: int = 1, intermediary: int = 0, on_image=None) -> SdImage:
        """One sample from padded [77] id rows (uncond = None: no classifier-free
        guidance; cond2 / uncond2: the second tokenizer's ids for xl / turbo).  img2img:
        init_latents [bsize, 4, h, w] (the encoded image scaled and noised to the schedule's
        step t_start, one noise draw per image) and the steps from t_start on.  bsize images per sample (init_noise then
        [bsize, 4, h, w]); intermediary > 0: on_image(step, rgb [n, H, W, 3]) after every
        step index divisible by it."""
        ids = [None if x is None else _ids(x).reshape(-1) for x in (cond, uncond, cond2, uncond2)]
        for x in ids:
            if x is not None and x.size != N_TOK:
                raise ValueError(f"id rows must be {N_TOK} long")
        bsize = max(1, int(bsize))
        noise = None if init_noise is None else _f32(init_noise).reshape(-1)
        h, w = self.height // 8, self.width // 8
        if noise is not None and noise.size != 4 * h * w * bsize:
            raise ValueError(f"init_noise must hold {4 * h * w * bsize} values")
        lat0 = None if init_latents is None else _f32(init_latents).reshape(-1)
        if lat0 is not None and lat0.size != 4 * h * w * bsize:
            raise ValueError(f"init_latents must hold {4 * h * w * bsize} values")
        err_cb: list = []

        def _cb(_ctx, step, n, ptr):
            try:
                arr = np.ctypeslib.as_array(ptr, shape=(n, self.height, self.width, 3)).copy()
                on_image(int(step), arr)
            except Exception as e:  # noqa: BLE001 - re-raised after the engine returns
                err_cb.append(e)
        cb = IMAGE_FN(_cb) if (on_image is not None and intermediary > 0) else None
        a = SdGenArgs(cond=_ip(ids[0]), uncond=_ip(ids[1]), cond2=_ip(ids[2]), uncond2=_ip(ids[3]),
                      n_steps=int(n_steps), guidance=float(guidance),
                      seed=int(seed) & 0xFFFFFFFFFFFFFFFF,
                      init_noise=None if noise is None else _fp(noise),
                      use_graph=1 if use_graph else 0, t_start=int(t_start),
                      init_latents=None if lat0 is None else _fp(lat0), bsize=bsize,
                      intermediary=int(intermediary) if cb is not None else 0,
                      on_image=C.cast(cb, C.c_void_p) if cb is not None else None, cb_ctx=None)
        n_run = int(n_steps) - (max(0, int(t_start)) if lat0 is not None else 0)
        rgb = np.empty((bsize, self.height, self.width, 3), dtype=np.uint8)
        lat = np.empty((bsize, 4, h, w), dtype=np.float32)
        steps = (C.c_double * max(1, n_run))()
        res = SdResult()
        err = C.create_string_buffer(1024)
        rc = lib().cake_sd_generate(self._h, C.byref(a), rgb.ctypes.data_as(C.POINTER(C.c_uint8)),
                                    _fp(lat), steps, C.byref(res), err, 1024)
        self._check(rc, err)
        if err_cb:
            raise err_cb[0]
        if bsize == 1:
            rgb, lat = rgb[0], lat[0]
        return SdImage(rgb, lat, [float(steps[i]) for i in range(n_run)], res.text_s,
                       res.denoise_s, res.vae_s)

    def text(self, which: int, ids) -> np.ndarray:
        """Text encoder `which` (0 CLIP, 1 the second encoder) on ids [B, 77] -> [B, 77, D]."""
        x = _ids(ids).reshape(-1, N_TOK)
        B = x.shape[0]
        D = self.text_dims[int(which)]
        if D == 0:
            raise ValueError("this version has one text encoder")
        out = np.empty((B, N_TOK, D), dtype=np.float32)
        err = C.create_string_buffer(1024)
        self._check(lib().cake_sd_text(self._h, int(which), _ip(x), B, _fp(out), err, 1024), err)
        return out

    def unet(self, sample, t: float, ctx) -> np.ndarray:
        """One UNet forward: sample [B, 4, h, w], ctx [B, 77, context_dim] -> [B, 4, h, w]."""
        s = _f32(sample)
        c = _f32(ctx)
        out = np.empty_like(s)
        err = C.create_string_buffer(1024)
        self._check(lib().cake_sd_unet(self._h, _fp(s), int(s.shape[0]), float(t), _fp(c),
                                       _fp(out), err, 1024), err)
        return out

    def vae_decode(self, z) -> np.ndarray:
        """z [1, 4, h, w] (already divided by vae_scale) -> image [1, 3, H, W] in [-1, 1]."""
        zz = _f32(z)
        img = np.empty((1, 3, self.height, self.width), dtype=np.float32)
        err = C.create_string_buffer(1024)
        self._check(lib().cake_sd_vae_decode(self._h, _fp(zz), _fp(img), err, 1024), err)
        return img

    def vae_encode(self, img) -> np.ndarray:
        """image [1, 3, H, W] in [-1, 1] -> posterior moments [1, 8, h, w] (mean | logvar)."""
        x = _f32(img)
        mo = np.empty((1, 8, self.height // 8, self.width // 8), dtype=np.float32)
        err = C.create_string_buffer(1024)
        self._check(lib().cake_sd_vae_encode(self._h, _fp(x), _fp(mo), err, 1024), err)
        return mo

    def vae_encode_remote(self, img) -> np.ndarray:
        """img2img with the topology's VAE worker: image [1, 3, H, W] -> the latent sample
        [1, 4, h, w] the worker draws (the Python client path's semantics)."""
        x = _f32(img)
        out = np.empty((1, 4, self.height // 8, self.width // 8), dtype=np.float32)
        err = C.create_string_buffer(1024)
        self._check(lib().cake_sd_vae_encode_remote(self._h, _fp(x), _fp(out), err, 1024), err)
        return out

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().cake_sd_close(self._h)
            self._h = None

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def native_sd_available() -> bool:
    return LIB_PATH.exists()
