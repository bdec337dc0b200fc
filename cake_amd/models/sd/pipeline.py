"""Stable Diffusion generator (cake-core/src/models/sd/sd.rs).

``load``: tokenizers (pad id = the config's ``pad_with`` token, else
``<|endoftext|>``), then each component — clip, clip2 (XL/Turbo), vae, unet —
either as a local unit or, when the topology names a worker for it, as a remote
unit over the framed protocol (component placement).

``generate_image``: defaults guidance 7.5 / steps 30 (Turbo: 0 / 1);
classifier-free guidance by batch doubling with [uncond, cond] embeddings;
XL/Turbo concatenate the two encoders' states on the last dim; ``bsize``
repeats the embeddings; img2img encodes the image, adds noise at
``t_start = n - floor(n * strength)``; every ``intermediary_images`` steps and
at the end the latents are decoded (``/ vae_scale``), mapped ``x/2 + 0.5``,
clamped and converted to 8-bit RGB images for the callback.  Per-step wall
time is logged (sd.rs:506-507) and, with ``tracing``, a chrome trace is
written to ``trace-<timestamp>.json`` (one file per request — Appendix E Q10).
"""
from __future__ import annotations

import logging
import math
import time
from pathlib import Path
from typing import Callable

import torch

from ..base import ImageGenerator
from ...utils.trace import ChromeTrace
from .args import ImageGenerationArgs
from .config import SDConfig
from .schedulers import build_scheduler
from .shardable import (RemoteSDUnit, load_unit, sd_config_for, unet_forward_unpacked, vae_decode,
                        vae_encode)
from .weights import resolve

log = logging.getLogger("cake.sd")


def image_preprocess(path: str) -> torch.Tensor:
    """Crop-resize to multiples of 32, map to [-1, 1], [1, 3, H, W] (sd.rs:647-665)."""
    from PIL import Image
    img = Image.open(path).convert("RGB")
    w, h = img.size
    w, h = w - w % 32, h - h % 32
    from PIL import ImageOps
    img = ImageOps.fit(img, (w, h), method=Image.BICUBIC)
    t = torch.frombuffer(bytearray(img.tobytes()), dtype=torch.uint8).reshape(h, w, 3)
    return (t.permute(2, 0, 1).float() * (2.0 / 255.0) - 1.0)[None]


def to_images(decoded: torch.Tensor) -> list:
    """[B, 3, H, W] in [-1, 1] -> 8-bit RGB PIL images (sd.rs:544-547): on the device
    path one kernel (sd_small.hip to_rgb8) writes u8 HWC, then one D2H copy."""
    from PIL import Image
    if decoded.is_cuda and decoded.dtype in (torch.float16, torch.bfloat16):
        from ...ops import hip as K
        x = K.to_rgb8(decoded.contiguous()).cpu()
    else:
        x = ((decoded.float() / 2 + 0.5).clamp(0, 1) * 255).to(torch.uint8).permute(0, 2, 3, 1)
        x = x.contiguous().cpu()
    return [Image.fromarray(x[b].numpy(), "RGB") for b in range(x.shape[0])]


class SDGenerator(ImageGenerator):
    MODEL_NAME = "stable-diffusion"

    def __init__(self, cfg: SDConfig, tokenizer, pad_id, text_model, vae, unet, device, dtype,
                 tokenizer_2=None, pad_id_2=None, text_model_2=None):
        self.cfg, self.device, self.dtype = cfg, device, dtype
        self.tokenizer, self.pad_id, self.text_model = tokenizer, pad_id, text_model
        self.tokenizer_2, self.pad_id_2, self.text_model_2 = tokenizer_2, pad_id_2, text_model_2
        self.vae, self.unet = vae, unet
        self.last_step_s: list[float] = []

    @classmethod
    def load(cls, ctx, remote=None) -> "SDGenerator":
        """remote(name) -> a proxy for a component served by another rank of a
        device-transport job (parallel/sd_rccl.py), or None; otherwise the topology
        decides between a local unit and a TCP worker."""
        from tokenizers import Tokenizer

        from ...parallel.client import Client
        a = ctx.args
        cfg = sd_config_for(ctx)
        xl = cfg.clip2 is not None

        def pad_of(tok, clip_cfg):
            p = clip_cfg.pad_with or "<|endoftext|>"
            pid = tok.token_to_id(p)
            if pid is None:
                raise ValueError(f"tokenizer has no pad token {p!r}")
            return pid

        tok = Tokenizer.from_file(str(resolve("tokenizer", a.sd_tokenizer, cfg.version, a.sd_use_f16,
                                              ctx.model_path)))
        tok2 = Tokenizer.from_file(str(resolve("tokenizer_2", a.sd_tokenizer_2, cfg.version,
                                               a.sd_use_f16, ctx.model_path))) if xl else None
        clients: dict[str, Client] = {}

        def component(name):
            if remote is not None:
                proxy = remote(name)
                if proxy is not None:
                    log.info("%s is served by %s", name, proxy.ident())
                    return proxy
                log.info("%s will be served locally", name)
                return load_unit(name, ctx, cfg)
            node = ctx.topology.get_node_for_layer(name)
            if node is not None:
                if node.name not in clients:
                    clients[node.name] = Client(ctx.device, node.host, name)
                log.info("node %s will serve %s", node.name, name)
                return RemoteSDUnit(clients[node.name], name)
            log.info("%s will be served locally", name)
            return load_unit(name, ctx, cfg)

        text_model = component("clip")
        text_model_2 = component("clip2") if xl else None
        vae = component("vae")
        unet = component("unet")
        return cls(cfg, tok, pad_of(tok, cfg.clip), text_model, vae, unet, ctx.device, ctx.dtype,
                   tok2, pad_of(tok2, cfg.clip2) if xl else None, text_model_2)

    # ------------------------------------------------------------------ text
    def _encode(self, tokenizer, pad_id, max_len, prompt: str) -> torch.Tensor:
        ids = tokenizer.encode(prompt, add_special_tokens=True).ids
        if len(ids) > max_len:
            raise ValueError(f"the prompt is too long, {len(ids)} > max-tokens ({max_len})")
        ids = ids + [pad_id] * (max_len - len(ids))
        return torch.tensor([ids], dtype=torch.int32, device=self.device)

    def text_embeddings(self, prompt: str, uncond: str, use_guide: bool, first: bool) -> torch.Tensor:
        if first:
            tok, model, pad, L = self.tokenizer, self.text_model, self.pad_id, \
                self.cfg.clip.max_position_embeddings
        else:
            tok, model, pad, L = self.tokenizer_2, self.text_model_2, self.pad_id_2, \
                self.cfg.clip2.max_position_embeddings
        log.info('Running with prompt "%s".', prompt)
        emb = model.forward(self._encode(tok, pad, L, prompt))
        if use_guide:
            u = model.forward(self._encode(tok, pad, L, uncond))
            emb = torch.cat([u.to(self.device), emb.to(self.device)], 0)
        return emb.to(device=self.device, dtype=self.dtype)

    def _fused_steps(self, intermediary: bool = False) -> bool:
        """Whole denoising loop as per-step graph replays: a local UNet, or one worker
        rank holding the entire UNet (device transport; the host needs no latents
        between steps unless intermediary images are requested)."""
        import os

        from .shardable import SDUnit
        local = isinstance(self.unet, SDUnit)
        if not (local or (getattr(self.unet, "can_denoise", False) and not intermediary)):
            return False
        return (torch.device(self.device).type == "cuda"
                and self.dtype in (torch.float16, torch.bfloat16)
                and os.environ.get("CAKE_SD_FUSED_STEP", "1") != "0")

    def _steps_eager(self, args, sched, ts, t_start, latents, text_emb, guidance, use_guide, gen,
                     trace, n_steps, callback):
        """One UNet round trip per step (remote UNet / CPU): the reference's loop."""
        for i, t in enumerate(ts):
            if i < t_start:
                continue
            t0 = time.perf_counter()
            with ChromeTrace.span(trace, f"step {i + 1}"):
                inp = torch.cat([latents, latents], 0) if use_guide else latents
                inp = sched.scale_model_input(inp, t)
                with ChromeTrace.span(trace, "unet"):
                    pred = unet_forward_unpacked(self.unet, inp.to(self.dtype), text_emb, t,
                                                 self.device).float()
                if use_guide:
                    u, c = pred.chunk(2, 0)
                    pred = u + (c - u) * guidance
                latents = sched.step(pred, t, latents, gen)
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            self.last_step_s.append(dt)
            log.info("step %d/%d done, %.2fs", i + 1, n_steps, dt)
            if args.intermediary_images and i % args.intermediary_images == 0:
                callback(self.split_images(latents))
        return latents

    # ------------------------------------------------------------------ images
    def split_images(self, latents: torch.Tensor) -> list:
        dec = vae_decode(self.vae, (latents / self.cfg.vae_scale).to(self.dtype), self.device)
        return to_images(dec)

    @torch.no_grad()
    def generate_image(self, args: ImageGenerationArgs, callback: Callable[[list], None]) -> None:
        cfg = self.cfg
        if not 0.0 <= args.img2img_strength <= 1.0:
            raise ValueError(f"img2img-strength should be between 0 and 1, got {args.img2img_strength}")
        trace = ChromeTrace() if args.tracing else None
        guidance = args.guidance_scale if args.guidance_scale is not None else cfg.default_guidance
        n_steps = args.n_steps if args.n_steps is not None else cfg.default_steps
        gen = torch.Generator(device="cpu")
        if args.image_seed is not None:
            gen.manual_seed(int(args.image_seed))
        else:
            gen.seed()
        use_guide = guidance > 1.0
        with ChromeTrace.span(trace, "text_embeddings"):
            embs = [self.text_embeddings(args.image_prompt, args.uncond_prompt, use_guide, True)]
            if cfg.clip2 is not None:
                embs.append(self.text_embeddings(args.image_prompt, args.uncond_prompt, use_guide, False))
            text_emb = torch.cat(embs, -1).repeat(args.bsize, 1, 1)
        init = None
        if args.img2img:
            img = image_preprocess(args.img2img).to(self.device, self.dtype)
            with ChromeTrace.span(trace, "vae_encode"):
                init = vae_encode(self.vae, img, self.device).float()
        t_start = n_steps - int(n_steps * args.img2img_strength) if args.img2img else 0
        sched = build_scheduler(cfg.scheduler, n_steps)
        self.last_step_s = []
        for idx in range(args.num_samples):
            ts = sched.timesteps()
            if init is not None:
                # bsize > 1: each image starts from the encoded image with its own noise
                # (the reference's latent stays batch 1 against bsize text rows)
                latents = init.repeat(args.bsize, 1, 1, 1) * cfg.vae_scale
                if t_start < len(ts):
                    noise = torch.randn(latents.shape, generator=gen).to(self.device)
                    latents = sched.add_noise(latents, noise, ts[t_start])
            else:
                shape = (args.bsize, 4, cfg.height // 8, cfg.width // 8)
                latents = torch.randn(shape, generator=gen).to(self.device) * sched.init_noise_sigma
            latents = latents.float()
            if self._fused_steps(bool(args.intermediary_images)) and t_start < len(ts):
                # local UNet on the GPU: each step is one graph replay (device timestep,
                # UNet, CFG + scheduler update + next input; SDUnit.denoise)
                steps = ts[t_start:]
                seed = int(torch.randint(0, 2 ** 62, (1,), generator=gen).item())

                def on_step(k, x, first=t_start):
                    i = first + k
                    if args.intermediary_images and i % args.intermediary_images == 0:
                        callback(self.split_images(x))
                with ChromeTrace.span(trace, f"denoise {len(steps)} steps"):
                    latents, dts = self.unet.denoise(
                        latents, text_emb, sched, steps, guidance, use_guide, seed,
                        on_step if args.intermediary_images else None)
                for k, dt in enumerate(dts):
                    self.last_step_s.append(dt)
                    log.info("step %d/%d done, %.2fs", t_start + k + 1, n_steps, dt)
            else:
                latents = self._steps_eager(args, sched, ts, t_start, latents, text_emb,
                                            guidance, use_guide, gen, trace, n_steps, callback)
            log.debug("Generating the final image for sample %d/%d.", idx + 1, args.num_samples)
            with ChromeTrace.span(trace, "vae_decode"):
                callback(self.split_images(latents))
        if trace is not None:
            path = Path(f"trace-{int(time.time() * 1000)}.json")
            trace.save(path)
            log.info("wrote chrome trace %s", path)
