"""Stable Diffusion configurations (the reference takes them from candle's
``StableDiffusionConfig::{v1_5, v2_1, sdxl, sdxl_turbo}``, cake-core/src/models/sd/sd.rs:134-149).

Architectures follow the diffusers checkpoints the reference downloads
(``runwayml/stable-diffusion-v1-5``, ``stabilityai/stable-diffusion-2-1``,
``stabilityai/stable-diffusion-xl-base-1.0``, ``stabilityai/sdxl-turbo``):
UNet2DConditionModel, AutoencoderKL, CLIP text encoders, DDIM / Euler-ancestral.
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class ClipConfig:
    vocab_size: int = 49408
    embed_dim: int = 768
    intermediate_size: int = 3072
    max_position_embeddings: int = 77
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    activation: str = "quick_gelu"   # or "gelu"
    pad_with: str | None = None      # None -> "<|endoftext|>"
    layer_norm_eps: float = 1e-5


@dataclass
class UNetBlock:
    out_channels: int
    cross_attn: bool
    heads: int               # attention heads of the block's transformers
    transformer_layers: int = 1


@dataclass
class UNetConfig:
    blocks: list[UNetBlock]
    in_channels: int = 4
    out_channels: int = 4
    layers_per_block: int = 2
    cross_attention_dim: int = 768
    use_linear_projection: bool = False
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    flip_sin_to_cos: bool = True
    freq_shift: float = 0.0
    sliced_attention_size: int | None = None


@dataclass
class VAEConfig:
    block_out_channels: tuple = (128, 256, 512, 512)
    layers_per_block: int = 2
    latent_channels: int = 4
    norm_num_groups: int = 32
    in_channels: int = 3
    out_channels: int = 3


@dataclass
class SchedulerConfig:
    kind: str = "ddim"                 # ddim | euler_ancestral
    beta_start: float = 0.00085
    beta_end: float = 0.012
    train_timesteps: int = 1000
    steps_offset: int = 1
    prediction_type: str = "epsilon"   # epsilon | v_prediction
    timestep_spacing: str = "leading"  # leading | trailing | linspace


@dataclass
class SDConfig:
    version: str
    width: int
    height: int
    unet: UNetConfig
    vae: VAEConfig
    clip: ClipConfig
    clip2: ClipConfig | None = None
    scheduler: SchedulerConfig = field(default_factory=SchedulerConfig)
    vae_scale: float = 0.18215
    default_guidance: float = 7.5
    default_steps: int = 30

    @property
    def context_dim(self) -> int:
        return self.clip.embed_dim + (self.clip2.embed_dim if self.clip2 else 0)


def _sd15_unet(sliced):
    return UNetConfig([UNetBlock(320, True, 8), UNetBlock(640, True, 8), UNetBlock(1280, True, 8),
                       UNetBlock(1280, False, 8)], cross_attention_dim=768,
                      sliced_attention_size=sliced)


def get_config(version: str, height: int | None = None, width: int | None = None,
               sliced_attention_size: int | None = None) -> SDConfig:
    """Version -> config; width/height default per version and must be multiples of 8."""
    v = version
    if v == "v1-5":
        cfg = SDConfig(v, 512, 512, _sd15_unet(sliced_attention_size), VAEConfig(), ClipConfig())
    elif v == "v2-1":
        unet = UNetConfig([UNetBlock(320, True, 5), UNetBlock(640, True, 10),
                           UNetBlock(1280, True, 20), UNetBlock(1280, False, 20)],
                          cross_attention_dim=1024, use_linear_projection=True,
                          sliced_attention_size=sliced_attention_size)
        clip = ClipConfig(embed_dim=1024, intermediate_size=4096, num_hidden_layers=23,
                          num_attention_heads=16, activation="gelu", pad_with="!")
        cfg = SDConfig(v, 768, 768, unet, VAEConfig(), clip,
                       scheduler=SchedulerConfig(prediction_type="v_prediction"))
    elif v in ("xl", "turbo"):
        unet = UNetConfig([UNetBlock(320, False, 5), UNetBlock(640, True, 10, 2),
                           UNetBlock(1280, True, 20, 10)], cross_attention_dim=2048,
                          use_linear_projection=True, sliced_attention_size=sliced_attention_size)
        clip = ClipConfig()
        clip2 = ClipConfig(embed_dim=1280, intermediate_size=5120, num_hidden_layers=32,
                           num_attention_heads=20, activation="gelu", pad_with="!")
        if v == "xl":
            cfg = SDConfig(v, 1024, 1024, unet, VAEConfig(), clip, clip2)
        else:
            cfg = SDConfig(v, 512, 512, unet, VAEConfig(), clip, clip2,
                           scheduler=SchedulerConfig(kind="euler_ancestral",
                                                     timestep_spacing="trailing"),
                           vae_scale=0.13025, default_guidance=0.0, default_steps=1)
    else:
        raise ValueError(f"unknown sd version {version!r} (v1-5, v2-1, xl, turbo)")
    if height is not None:
        cfg.height = height
    if width is not None:
        cfg.width = width
    if cfg.height % 8 or cfg.width % 8:
        raise ValueError(f"height/width must be multiples of 8, got {cfg.height}x{cfg.width}")
    return cfg


def tiny_config(version: str = "v1-5") -> SDConfig:
    """A structurally complete, small SD for tests (same block types as the real ones)."""
    xl = version in ("xl", "turbo")
    if xl:
        unet = UNetConfig([UNetBlock(32, False, 2), UNetBlock(64, True, 2, 2)],
                          cross_attention_dim=64, use_linear_projection=True, norm_num_groups=8)
        clip = ClipConfig(vocab_size=512, embed_dim=32, intermediate_size=64, num_hidden_layers=2,
                          num_attention_heads=2)
        clip2 = ClipConfig(vocab_size=512, embed_dim=32, intermediate_size=64, num_hidden_layers=2,
                           num_attention_heads=2, activation="gelu", pad_with="!")
    else:
        unet = UNetConfig([UNetBlock(32, True, 4), UNetBlock(64, True, 4), UNetBlock(64, False, 4)],
                          cross_attention_dim=32, norm_num_groups=8,
                          use_linear_projection=version == "v2-1")
        clip = ClipConfig(vocab_size=512, embed_dim=32, intermediate_size=64, num_hidden_layers=2,
                          num_attention_heads=2)
        clip2 = None
    vae = VAEConfig(block_out_channels=(16, 16, 32, 32), layers_per_block=1, norm_num_groups=8)
    base = get_config(version)
    return SDConfig(version, 64, 64, unet, vae, clip, clip2, scheduler=base.scheduler,
                    vae_scale=base.vae_scale, default_guidance=base.default_guidance,
                    default_steps=base.default_steps)


def mini_config(version: str = "v1-5") -> SDConfig:
    """A small SD whose every shape takes the HIP kernel paths (channel counts multiples
    of 64, GroupNorm groups of >= 4 channels; tiny_config's 32-channel convolutions fall
    back to the library there): the native engine's parity tests
    (csrc/engine/sd_engine.cpp reads the same architecture from cake_sd.json)."""
    if version in ("xl", "turbo"):
        unet = UNetConfig([UNetBlock(64, False, 2), UNetBlock(128, True, 2, 2)],
                          cross_attention_dim=128, use_linear_projection=True, norm_num_groups=16)
        clip = ClipConfig(vocab_size=512, embed_dim=64, intermediate_size=128, num_hidden_layers=2,
                          num_attention_heads=2)
        clip2 = ClipConfig(vocab_size=512, embed_dim=64, intermediate_size=128, num_hidden_layers=2,
                           num_attention_heads=2, activation="gelu", pad_with="!")
    else:
        unet = UNetConfig([UNetBlock(64, True, 2), UNetBlock(128, True, 2),
                           UNetBlock(128, False, 2)], cross_attention_dim=64, norm_num_groups=16,
                          use_linear_projection=version == "v2-1")
        clip = ClipConfig(vocab_size=512, embed_dim=64, intermediate_size=128, num_hidden_layers=2,
                          num_attention_heads=2)
        clip2 = None
    vae = VAEConfig(block_out_channels=(64, 64, 128, 128), layers_per_block=1, norm_num_groups=16)
    base = get_config(version)
    return SDConfig(version, 64, 64, unet, vae, clip, clip2, scheduler=base.scheduler,
                    vae_scale=base.vae_scale, default_guidance=base.default_guidance,
                    default_steps=base.default_steps)
