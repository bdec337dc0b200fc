"""Image generation arguments (cake-core/src/lib.rs:129-200 ``ImageGenerationArgs``).

The same struct is filled from the CLI (``--sd-*`` flags) and from the image
API JSON (``image_args`` object with the same ``sd-*`` kebab-case keys and the
serde defaults: prompt = rusty robot, uncond = "", num_samples = 1, bsize = 1,
img2img_strength = 0.8, everything else unset/0).
"""
from __future__ import annotations

from dataclasses import dataclass

DEFAULT_PROMPT = "A very realistic photo of a rusty robot walking on a sandy beach"


@dataclass
class ImageGenerationArgs:
    image_prompt: str = DEFAULT_PROMPT
    uncond_prompt: str = ""
    tracing: bool = False
    n_steps: int | None = None
    num_samples: int = 1
    bsize: int = 1
    intermediary_images: int = 0
    guidance_scale: float | None = None
    img2img: str | None = None
    img2img_strength: float = 0.8
    image_seed: int | None = None

    @classmethod
    def from_cli(cls, a) -> "ImageGenerationArgs":
        return cls(image_prompt=a.sd_image_prompt, uncond_prompt=a.sd_uncond_prompt,
                   tracing=a.sd_tracing, n_steps=a.sd_n_steps, num_samples=a.sd_num_samples,
                   bsize=a.sd_bsize, intermediary_images=a.sd_intermediary_images,
                   guidance_scale=a.sd_guidance_scale, img2img=a.sd_img2img,
                   img2img_strength=a.sd_img2img_strength, image_seed=a.sd_seed)

    @classmethod
    def from_json(cls, d: dict) -> "ImageGenerationArgs":
        g = d.get
        return cls(image_prompt=g("sd-image-prompt", DEFAULT_PROMPT),
                   uncond_prompt=g("sd-uncond-prompt", ""), tracing=bool(g("sd-tracing", False)),
                   n_steps=g("sd-n-steps"), num_samples=int(g("sd-num-samples", 1)),
                   bsize=int(g("sd-bsize", 1)),
                   intermediary_images=int(g("sd-intermediary-images", 0)),
                   guidance_scale=g("sd-guidance-scale"), img2img=g("sd-img2img"),
                   img2img_strength=float(g("sd-img2img-strength", 0.8)),
                   image_seed=g("sd-seed"))
