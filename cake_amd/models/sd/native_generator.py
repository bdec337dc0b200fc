"""Stable Diffusion generator on the native engine (csrc/engine/sd_engine.cpp).

The reference's generate_image (cake-core/src/models/sd/sd.rs:320-532) behind the
ImageGenerator contract with the whole generation in C++ — both text encoders, the
guided denoising loop (graph replays) and the VAE decode; the tokenizers (HF
``tokenizers``), the seeded latent noise and the PNG writing stay here.  The noise and
the ancestral-noise key are drawn from the request's generator in the same order as the
Python pipeline (models/sd/pipeline.py), so a seed gives the same image on either path.

img2img runs natively too: the engine encodes the image (VAE encoder), the posterior
sample, the latent scaling and the noise to the start step are drawn here with the same
generators and torch ops as the Python pipeline, and the engine denoises from that step.
bsize > 1 (the UNet over 2 bsize rows, the reference's repeated text rows), intermediary
images (decoded by the engine between steps, handed back through a callback) and tracing
(the Chrome trace spans — text embeddings, every step, VAE decode — rebuilt from the
engine's own phase and per-step device timings) are native (img2img with a remote VAE
too: the worker encodes and draws the sample; img2img at bsize > 1 starts every image from
the encoded image with its own noise draw, as pipeline.py does).  Only an img2img image
whose size is not the engine's runs on the Python pipeline, built on first use.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Callable

import numpy as np
import torch

from ..base import ImageGenerator
from .args import ImageGenerationArgs
from .config import SDConfig
from .weights import resolve

log = logging.getLogger("cake.sd")


class NativeSDGenerator(ImageGenerator):
    MODEL_NAME = "stable-diffusion"

    def __init__(self, cfg: SDConfig, engine, tok, pad_id, tok2=None, pad_id2=None,
                 fallback: Callable[[], ImageGenerator] | None = None):
        self.cfg, self.eng = cfg, engine
        self.tok, self.pad_id, self.tok2, self.pad_id2 = tok, pad_id, tok2, pad_id2
        self._fallback_factory = fallback
        self._fallback = None
        # the VAE unit's own posterior-sampling generator (shardable.SDUnit.generator)
        self.vae_generator = torch.Generator(device="cpu")
        self.last_step_s: list[float] = []
        self.last_result = None

    @classmethod
    def load(cls, ctx, split: dict | None = None) -> "NativeSDGenerator":
        """split: rank 0 of a native split UNet (NativeSD rank / world / master_addr /
        owners keyword arguments; parallel/sd_rccl.py run_native_split)."""
        from tokenizers import Tokenizer

        from ...sd_engine import NativeSD
        from .shardable import sd_config_for
        a = ctx.args
        cfg = sd_config_for(ctx)
        xl = cfg.clip2 is not None

        def pad_of(tok, clip_cfg):
            pid = tok.token_to_id(clip_cfg.pad_with or "<|endoftext|>")
            if pid is None:
                raise ValueError(f"tokenizer has no pad token {clip_cfg.pad_with!r}")
            return pid
        tok = Tokenizer.from_file(str(resolve("tokenizer", a.sd_tokenizer, cfg.version, a.sd_use_f16,
                                              ctx.model_path)))
        tok2 = Tokenizer.from_file(str(resolve("tokenizer_2", a.sd_tokenizer_2, cfg.version,
                                               a.sd_use_f16, ctx.model_path))) if xl else None
        paths, remote = {}, {}
        topo = getattr(ctx, "topology", None)
        for comp, flag in (("unet", "sd_unet"), ("vae", "sd_vae"), ("clip", "sd_clip"),
                           ("clip2", "sd_clip2")):
            if comp == "clip2" and not xl:
                continue
            node = topo.get_node_for_layer(comp) if topo is not None else None
            if node is not None:  # served by a TCP worker (sd.rs: the topology's component)
                remote[comp] = node.host
                continue
            paths[comp] = str(resolve(comp, getattr(a, flag, None), cfg.version, a.sd_use_f16,
                                      ctx.model_path))
        eng = NativeSD(str(ctx.model_path), version=cfg.version, width=cfg.width,
                       height=cfg.height, dtype="bf16" if ctx.dtype == torch.bfloat16 else "f16",
                       device=ctx.device.index or 0, paths=paths, remote=remote, **(split or {}))

        def fallback():
            from .pipeline import SDGenerator
            return SDGenerator.load(ctx)
        return cls(cfg, eng, tok, pad_of(tok, cfg.clip), tok2,
                   pad_of(tok2, cfg.clip2) if xl else None, fallback)

    def _ids(self, tok, pad, prompt: str) -> np.ndarray:
        ids = tok.encode(prompt, add_special_tokens=True).ids
        if len(ids) > 77:
            raise ValueError(f"the prompt is too long, {len(ids)} > max-tokens (77)")
        return np.asarray(ids + [pad] * (77 - len(ids)), dtype=np.int32)

    def _python(self) -> ImageGenerator:
        if self._fallback is None:
            log.info("request needs the Python pipeline (an img2img image of another size)")
            self._fallback = self._fallback_factory()
        return self._fallback

    def _encode_image(self, path: str):
        """pipeline.py image_preprocess + vae_encode on the engine: the latent sample
        [1, 4, h, w] (model dtype, as the Python VAE unit returns it), or None when the
        image does not have the engine's resolution."""
        from .pipeline import image_preprocess
        img = image_preprocess(path)
        if tuple(img.shape[2:]) != (self.cfg.height, self.cfg.width):
            return None
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        dt = torch.bfloat16 if self.eng._dt == 0 else torch.float16
        if "vae" in self.eng.remote:  # the worker encodes and draws the sample
            x = img.to(dt).float().numpy()  # the model-dtype image the client path sends
            return torch.from_numpy(self.eng.vae_encode_remote(x)).to(dev).to(dt)
        mo = torch.from_numpy(self.eng.vae_encode(img.numpy()))
        moments = mo.to(dev).to(dt).float()
        mean, logvar = moments.chunk(2, 1)
        logvar = logvar.clamp(-30.0, 20.0)
        eps = torch.randn(mean.shape, generator=self.vae_generator, device="cpu").to(mean.device)
        return (mean + torch.exp(0.5 * logvar) * eps).to(dt)

    def generate_image(self, args: ImageGenerationArgs, callback: Callable[[list], None]) -> None:
        init = None
        if args.img2img:
            if not 0.0 <= args.img2img_strength <= 1.0:
                raise ValueError("img2img-strength should be between 0 and 1, got "
                                 f"{args.img2img_strength}")
            init = self._encode_image(args.img2img)
        if args.img2img and init is None:
            gen = self._python()
            gen.generate_image(args, callback)
            self.last_step_s = list(getattr(gen, "last_step_s", []))
            return
        from PIL import Image
        cfg = self.cfg
        guidance = args.guidance_scale if args.guidance_scale is not None else cfg.default_guidance
        n_steps = args.n_steps if args.n_steps is not None else cfg.default_steps
        gen = torch.Generator(device="cpu")
        if args.image_seed is not None:
            gen.manual_seed(int(args.image_seed))
        else:
            gen.seed()
        use_guide = guidance > 1.0
        kw = {"cond": self._ids(self.tok, self.pad_id, args.image_prompt)}
        if use_guide:
            kw["uncond"] = self._ids(self.tok, self.pad_id, args.uncond_prompt)
        if self.tok2 is not None:
            kw["cond2"] = self._ids(self.tok2, self.pad_id2, args.image_prompt)
            if use_guide:
                kw["uncond2"] = self._ids(self.tok2, self.pad_id2, args.uncond_prompt)
        log.info('Running with prompt "%s".', args.image_prompt)
        self.last_step_s = []
        bsize = max(1, int(args.bsize))

        def pil(rgb: np.ndarray) -> list:
            rgb = rgb.reshape(-1, cfg.height, cfg.width, 3)
            return [Image.fromarray(np.ascontiguousarray(x), "RGB") for x in rgb]
        every = int(args.intermediary_images or 0)
        mid = {"intermediary": every, "on_image": (lambda _step, rgb: callback(pil(rgb)))} \
            if every > 0 else {}
        t_start = n_steps - int(n_steps * args.img2img_strength) if init is not None else 0
        trace = None
        if args.tracing:
            from ...utils.trace import ChromeTrace
            trace = ChromeTrace()
        for idx in range(args.num_samples):
            t0 = time.perf_counter()
            if init is not None:  # pipeline.py's img2img latents, same draws and ops
                from .schedulers import build_scheduler
                sched = build_scheduler(cfg.scheduler, n_steps)
                ts = sched.timesteps()
                # bsize > 1: every image starts from the encoded image, each with its own
                # noise draw (pipeline.py repeats the latent the same way)
                latents = init.float().repeat(bsize, 1, 1, 1) * cfg.vae_scale
                if t_start < len(ts):
                    noise = torch.randn(latents.shape, generator=gen).to(latents.device)
                    latents = sched.add_noise(latents, noise, ts[t_start])
                latents = latents.float()
                if t_start >= len(ts):  # strength 0: the encoded image itself
                    img = self.eng.vae_decode((latents[:1] / cfg.vae_scale).cpu().numpy())
                    rgb = ((np.clip(img[0] / 2 + 0.5, 0, 1) * 255).astype(np.uint8)
                           .transpose(1, 2, 0).copy())
                    callback([Image.fromarray(rgb, "RGB")] * bsize)
                    continue
                seed = int(torch.randint(0, 2 ** 62, (1,), generator=gen).item())
                out = self.eng.generate(n_steps=n_steps, guidance=guidance, seed=seed,
                                        init_latents=latents.cpu().numpy(), t_start=t_start,
                                        bsize=bsize, **kw, **mid)
            else:
                # the Python pipeline's draw order: latent noise, then the ancestral-noise key
                noise = torch.randn((bsize, 4, cfg.height // 8, cfg.width // 8), generator=gen)
                seed = int(torch.randint(0, 2 ** 62, (1,), generator=gen).item())
                out = self.eng.generate(n_steps=n_steps, guidance=guidance, seed=seed,
                                        init_noise=noise.numpy(), bsize=bsize, **kw, **mid)
            self.last_result = out
            if trace is not None:  # the pipeline's spans, from the engine's timings
                t_end = time.perf_counter()
                ts0 = t_end - (out.text_s + out.denoise_s + out.vae_s)
                trace.add("text_embeddings", ts0, ts0 + out.text_s)
                cur = ts0 + out.text_s
                trace.add(f"denoise {len(out.step_s)} steps", cur, cur + out.denoise_s)
                for k, dt in enumerate(out.step_s):
                    trace.add(f"step {t_start + k + 1}", cur, cur + dt, device_s=dt)
                    cur += dt
                trace.add("vae_decode", t_end - out.vae_s, t_end, images=bsize)
            for k, dt in enumerate(out.step_s):
                self.last_step_s.append(dt)
                log.info("step %d/%d done, %.2fs", t_start + k + 1, n_steps, dt)
            log.info("sample %d/%d: text %.1f ms, denoise %.1f ms, vae %.1f ms (%.1f ms total)",
                     idx + 1, args.num_samples, out.text_s * 1e3, out.denoise_s * 1e3,
                     out.vae_s * 1e3, (time.perf_counter() - t0) * 1e3)
            callback(pil(out.rgb))
        if trace is not None:
            from pathlib import Path
            path = Path(f"trace-{int(time.time() * 1000)}.json")
            trace.save(path)
            log.info("wrote chrome trace %s", path)


def native_sd_eligible(ctx) -> bool:
    """A GPU master, a 16-bit dtype, CAKE_NATIVE != 0, engine built (components local or
    served by the topology's workers)."""
    if os.environ.get("CAKE_NATIVE", "1") == "0":
        return False
    if ctx.device.type != "cuda" or ctx.dtype not in (torch.float16, torch.bfloat16):
        return False
    # components in the topology are served by their TCP workers through the engine's
    # client (remote_unet / _vae / _clip / _clip2)
    if getattr(ctx.args, "sd_sliced_attention_size", None):
        return True  # (flash attention has no score memory to slice)
    from ...sd_engine import native_sd_available
    return native_sd_available()
