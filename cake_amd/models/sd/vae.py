"""AutoencoderKL (diffusers layout; candle ``build_vae`` in the reference,
cake-core/src/models/sd/vae.rs).

encode: encoder → quant_conv → (mean, logvar) → mean + exp(logvar/2)·ε
decode: post_quant_conv → decoder (mid-block single-head attention, resnets,
nearest-2x upsampling) → RGB in [-1, 1].
The mid-block attention has one head of dim C (512): q|k|v is one fused GEMM,
the attention is the head-dim-512 MFMA flash kernel (attn512.hip; the
generic flash kernel for C <= 256), and the output projection adds the block
residual in its GEMM epilogue.
Accepts both current (to_q/to_k/to_v/to_out.0) and legacy
(query/key/value/proj_attn) attention weight names.
"""
from __future__ import annotations

import torch

from . import ops
from .config import VAEConfig
from .unet import Conv, Linear, Module, Norm, ResnetBlock2D

_LEGACY = {"to_q": "query", "to_k": "key", "to_v": "value", "to_out.0": "proj_attn"}


def normalize_vae_weights(w: dict[str, torch.Tensor]) -> dict[str, torch.Tensor]:
    out = {}
    for k, v in w.items():
        nk = k
        for new, old in _LEGACY.items():
            if f".attentions.0.{old}." in k:
                nk = k.replace(f".attentions.0.{old}.", f".attentions.0.{new}.")
        if nk.endswith((".to_q.weight", ".to_k.weight", ".to_v.weight", ".to_out.0.weight")) \
                and v.dim() == 4:  # 1x1 conv form
            v = v[:, :, 0, 0]
        out[nk] = v
    return out


class VAEAttention(Module):
    def __init__(self, name, ch, groups):
        self.name, self.groups = name, groups
        self.norm = Norm(f"{name}.group_norm", ch)
        self.q, self.k, self.v = (Linear(f"{name}.{n}", ch, ch) for n in ("to_q", "to_k", "to_v"))
        self.o = Linear(f"{name}.to_out.0", ch, ch)

    def params(self):
        p = {}
        for m in (self.norm, self.q, self.k, self.v, self.o):
            p.update(m.params())
        return p

    def __call__(self, W, x):
        h = ops.group_norm(x, W[f"{self.name}.group_norm.weight"], W[f"{self.name}.group_norm.bias"],
                           self.groups, 1e-6)
        h = ops.tokens(h)
        C = self.q.cout
        key = f"{self.name}.qkv@fused"
        if key not in W:
            W[key] = torch.cat([W[f"{self.name}.{n}.weight"] for n in ("to_q", "to_k", "to_v")], 0)
            W[key + ".bias"] = torch.cat([W[f"{self.name}.{n}.bias"]
                                          for n in ("to_q", "to_k", "to_v")], 0)
        qkv = ops.linear(h, W[key], W[key + ".bias"])  # one GEMM for q|k|v
        a = ops.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], 1)
        if ops.nhwc():  # residual fused into the output projection's epilogue
            return ops.untokens(self.o(W, a, resid=ops.tokens(x)), x)
        return ops.untokens(self.o(W, a), x) + x


class AutoencoderKL(Module):
    def __init__(self, cfg: VAEConfig):
        self.cfg = cfg
        ch = list(cfg.block_out_channels)
        G = cfg.norm_num_groups
        L = cfg.layers_per_block
        # encoder
        self.e_in = Conv("encoder.conv_in", cfg.in_channels, ch[0])
        self.e_down = []
        out = ch[0]
        for i, c in enumerate(ch):
            cin, out = out, c
            res = [ResnetBlock2D(f"encoder.down_blocks.{i}.resnets.{j}", cin if j == 0 else out, out,
                                 0, G, 1e-6) for j in range(L)]
            ds = None if i == len(ch) - 1 else Conv(f"encoder.down_blocks.{i}.downsamplers.0.conv",
                                                    out, out, 3, 2, 0)
            self.e_down.append((res, ds))
        self.e_mid = [ResnetBlock2D(f"encoder.mid_block.resnets.{j}", ch[-1], ch[-1], 0, G, 1e-6)
                      for j in (0, 1)]
        self.e_att = VAEAttention("encoder.mid_block.attentions.0", ch[-1], G)
        self.e_norm = Norm("encoder.conv_norm_out", ch[-1])
        self.e_out = Conv("encoder.conv_out", ch[-1], 2 * cfg.latent_channels)
        self.quant = Conv("quant_conv", 2 * cfg.latent_channels, 2 * cfg.latent_channels, 1, 1, 0)
        # decoder
        self.post_quant = Conv("post_quant_conv", cfg.latent_channels, cfg.latent_channels, 1, 1, 0)
        self.d_in = Conv("decoder.conv_in", cfg.latent_channels, ch[-1])
        self.d_mid = [ResnetBlock2D(f"decoder.mid_block.resnets.{j}", ch[-1], ch[-1], 0, G, 1e-6)
                      for j in (0, 1)]
        self.d_att = VAEAttention("decoder.mid_block.attentions.0", ch[-1], G)
        self.d_up = []
        rev = list(reversed(ch))
        out = rev[0]
        for i, c in enumerate(rev):
            prev, out = out, c
            res = [ResnetBlock2D(f"decoder.up_blocks.{i}.resnets.{j}", prev if j == 0 else out, out,
                                 0, G, 1e-6) for j in range(L + 1)]
            us = None if i == len(ch) - 1 else Conv(f"decoder.up_blocks.{i}.upsamplers.0.conv", out, out)
            self.d_up.append((res, us))
        self.d_norm = Norm("decoder.conv_norm_out", ch[0])
        self.d_out = Conv("decoder.conv_out", ch[0], cfg.out_channels)

    def params(self):
        mods = [self.e_in, *self.e_mid, self.e_att, self.e_norm, self.e_out, self.quant,
                self.post_quant, self.d_in, *self.d_mid, self.d_att, self.d_norm, self.d_out]
        for res, s in self.e_down + self.d_up:
            mods += res + ([s] if s else [])
        p = {}
        for m in mods:
            p.update(m.params())
        return p

    def encode(self, W, x: torch.Tensor, generator: torch.Generator | None = None) -> torch.Tensor:
        """image [B,3,H,W] in [-1,1] -> latent sample [B,4,H/8,W/8] (unscaled)."""
        with ops.layout_nhwc(ops.want_nhwc(x)):
            moments = self._encode(W, x).float()
        mean, logvar = moments.chunk(2, 1)
        logvar = logvar.clamp(-30.0, 20.0)
        eps = torch.randn(mean.shape, generator=generator, device="cpu").to(mean.device)
        return (mean + torch.exp(0.5 * logvar) * eps).to(x.dtype)

    def _encode(self, W, x):
        """x: the external NCHW image; returns the NCHW moments (the first and last
        convolutions read / write that layout themselves)."""
        G = self.cfg.norm_num_groups
        h = self.e_in(W, x, in_nchw=True)
        for res, ds in self.e_down:
            for r in res:
                h = r(W, h)
            if ds is not None:
                h = ds(W, ops.pad_hw_end(h))
        h = self.e_mid[0](W, h)
        h = self.e_att(W, h)
        h = self.e_mid[1](W, h)
        h = ops.group_norm(h, W["encoder.conv_norm_out.weight"], W["encoder.conv_norm_out.bias"],
                           G, 1e-6, silu=True)
        return self.quant(W, self.e_out(W, h), out_nchw=True)

    def decode(self, W, z: torch.Tensor) -> torch.Tensor:
        with ops.layout_nhwc(ops.want_nhwc(z)):
            return self._decode(W, z)

    def _decode(self, W, z):
        """z: the external NCHW latent; returns the NCHW image (post_quant_conv reads and
        decoder.conv_out writes that layout themselves: no layout-copy kernels)."""
        G = self.cfg.norm_num_groups
        h = self.d_in(W, self.post_quant(W, z, in_nchw=True))
        h = self.d_mid[0](W, h)
        h = self.d_att(W, h)
        h = self.d_mid[1](W, h)
        for res, us in self.d_up:
            for r in res:
                h = r(W, h)
            if us is not None:
                h = us(W, h, up=True)
        h = ops.group_norm(h, W["decoder.conv_norm_out.weight"], W["decoder.conv_norm_out.bias"],
                           G, 1e-6, silu=True)
        return self.d_out(W, h, out_nchw=True)
