"""UNet2DConditionModel (diffusers layout; candle ``build_unet`` in the reference,
cake-core/src/models/sd/unet.rs:67-79).

Structure: conv_in → timestep embedding (sinusoidal, flip_sin_to_cos) →
down blocks [ResnetBlock2D (+ Transformer2DModel)]* (+ stride-2 conv) →
mid block (resnet, transformer, resnet) → up blocks with skip concatenation
(+ nearest-2x upsample conv) → GroupNorm/SiLU/conv_out.  SDXL's added
text-time conditioning is NOT used (cake passes only encoder_hidden_states,
unet.rs:54), matching the reference.

Each module is built once from the config and knows both its parameter
shapes (for random init / checkpoint validation) and its forward.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import ops
from .config import UNetConfig


class Module:
    def params(self) -> dict[str, tuple]:
        raise NotImplementedError


class Conv(Module):
    def __init__(self, name, cin, cout, k=3, stride=1, padding=None, bias=True):
        self.name, self.cin, self.cout, self.k, self.stride = name, cin, cout, k, stride
        self.padding = (k // 2) if padding is None else padding
        self.bias = bias

    def params(self):
        p = {f"{self.name}.weight": (self.cout, self.cin, self.k, self.k)}
        if self.bias:
            p[f"{self.name}.bias"] = (self.cout,)
        return p

    def __call__(self, W, x, up=False, bias2=None, resid=None, in_nchw=False, out_nchw=False):
        return ops.conv(W, self.name, x, self.stride, self.padding, up=up, bias2=bias2,
                        resid=resid, in_nchw=in_nchw, out_nchw=out_nchw)


class Linear(Module):
    def __init__(self, name, cin, cout, bias=True):
        self.name, self.cin, self.cout, self.bias = name, cin, cout, bias

    def params(self):
        p = {f"{self.name}.weight": (self.cout, self.cin)}
        if self.bias:
            p[f"{self.name}.bias"] = (self.cout,)
        return p

    def __call__(self, W, x, resid=None, gated=None):
        return ops.linear(x, W[f"{self.name}.weight"], W.get(f"{self.name}.bias"), resid=resid,
                          gated=gated)


class Norm(Module):
    def __init__(self, name, c):
        self.name, self.c = name, c

    def params(self):
        return {f"{self.name}.weight": (self.c,), f"{self.name}.bias": (self.c,)}


class ResnetBlock2D(Module):
    def __init__(self, name, cin, cout, temb_dim, groups, eps):
        self.name, self.cin, self.cout, self.groups, self.eps = name, cin, cout, groups, eps
        self.norm1 = Norm(f"{name}.norm1", cin)
        self.conv1 = Conv(f"{name}.conv1", cin, cout)
        self.temb = Linear(f"{name}.time_emb_proj", temb_dim, cout) if temb_dim else None
        self.norm2 = Norm(f"{name}.norm2", cout)
        self.conv2 = Conv(f"{name}.conv2", cout, cout)
        self.short = Conv(f"{name}.conv_shortcut", cin, cout, k=1, padding=0) if cin != cout else None

    def params(self):
        p = {}
        for m in (self.norm1, self.conv1, self.temb, self.norm2, self.conv2, self.short):
            if m is not None:
                p.update(m.params())
        return p

    def __call__(self, W, x, temb=None, tb=None, skip=None):
        """temb: the time embedding (the block projects silu(temb) itself), or tb: this
        block's precomputed time bias [B, C_out] f32 (the UNet batches every block's
        projection into one GEMM).  skip: the up path's skip tensor; the block input
        is then the channel concatenation [x, skip], formed inside norm1."""
        if skip is not None:
            h, x = ops.group_norm_cat(x, skip, W[f"{self.name}.norm1.weight"],
                                      W[f"{self.name}.norm1.bias"], self.groups, self.eps,
                                      silu=True, want_cat=True)
        else:
            h = ops.group_norm(x, W[f"{self.name}.norm1.weight"], W[f"{self.name}.norm1.bias"],
                               self.groups, self.eps, silu=True)
        if tb is None and self.temb is not None and temb is not None:
            tb = self.temb(W, F.silu(temb))
        h = self.conv1(W, h, bias2=tb)  # time embedding fused as a per-sample bias
        h = ops.group_norm(h, W[f"{self.name}.norm2.weight"], W[f"{self.name}.norm2.bias"],
                           self.groups, self.eps, silu=True)
        short = self.short(W, x) if self.short is not None else x
        return self.conv2(W, h, resid=short)  # residual fused into the epilogue


class Attention(Module):
    """diffusers Attention: to_q/to_k/to_v (no bias), to_out.0 (bias)."""

    def __init__(self, name, dim, ctx_dim, heads, sliced=None):
        self.name, self.heads, self.sliced = name, heads, sliced
        self.q = Linear(f"{name}.to_q", dim, dim, bias=False)
        self.k = Linear(f"{name}.to_k", ctx_dim, dim, bias=False)
        self.v = Linear(f"{name}.to_v", ctx_dim, dim, bias=False)
        self.o = Linear(f"{name}.to_out.0", dim, dim)

    def params(self):
        p = {}
        for m in (self.q, self.k, self.v, self.o):
            p.update(m.params())
        return p

    def _fused(self, W, names):
        key = f"{self.name}.{'+'.join(names)}@fused"
        w = W.get(key)
        if w is None:
            w = W[key] = torch.cat([W[f"{self.name}.{n}.weight"] for n in names], 0)
        return w

    def __call__(self, W, x, ctx=None, kv_cache=None, resid=None):
        C = self.q.cout
        if ctx is None:  # self-attention: one GEMM for q, k and v
            qkv = ops.linear(x, self._fused(W, ("to_q", "to_k", "to_v")))
            q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        else:
            # cross-attention: k/v depend only on the text context, which is fixed
            # for a whole generation -> computed once per context (kv_cache)
            q = self.q(W, x)
            kv = kv_cache.get(self.name) if kv_cache is not None else None
            if kv is None:
                wkv = self._fused(W, ("to_k", "to_v"))
                kv = ops.linear(ctx, wkv)
                if kv_cache is not None:
                    kv_cache[self.name] = kv
                    kv_cache[f"{self.name}@w"] = wkv
            k, v = kv[..., :C], kv[..., C:]
        a = ops.attention(q, k, v, self.heads, sliced=self.sliced)
        return self.o(W, a, resid=resid)  # + residual in the GEMM epilogue


class BasicTransformerBlock(Module):
    def __init__(self, name, dim, ctx_dim, heads, sliced):
        self.name = name
        self.n1, self.n2, self.n3 = (Norm(f"{name}.norm{i}", dim) for i in (1, 2, 3))
        self.attn1 = Attention(f"{name}.attn1", dim, dim, heads, sliced)
        self.attn2 = Attention(f"{name}.attn2", dim, ctx_dim, heads, sliced)
        self.ff_in = Linear(f"{name}.ff.net.0.proj", dim, dim * 8)  # GEGLU: 2 x 4*dim
        self.ff_out = Linear(f"{name}.ff.net.2", dim * 4, dim)

    def params(self):
        p = {}
        for m in (self.n1, self.n2, self.n3, self.attn1, self.attn2, self.ff_in, self.ff_out):
            p.update(m.params())
        return p

    def __call__(self, W, x, ctx, kv_cache=None):
        n = self.name
        x = self.attn1(W, ops.layer_norm(x, W[f"{n}.norm1.weight"], W[f"{n}.norm1.bias"], 1e-5),
                       resid=x)
        x = self.attn2(W, ops.layer_norm(x, W[f"{n}.norm2.weight"], W[f"{n}.norm2.bias"], 1e-5),
                       ctx, kv_cache, resid=x)
        h = ops.layer_norm(x, W[f"{n}.norm3.weight"], W[f"{n}.norm3.bias"], 1e-5)
        # GEGLU fused into the FF input projection, residual into the output projection
        return self.ff_out(W, self.ff_in(W, h, gated="geglu"), resid=x)


class Transformer2DModel(Module):
    """SpatialTransformer: GroupNorm → proj_in → blocks → proj_out → + residual."""

    def __init__(self, name, ch, ctx_dim, heads, layers, linear_proj, groups, sliced):
        self.name, self.ch, self.groups, self.linear = name, ch, groups, linear_proj
        self.norm = Norm(f"{name}.norm", ch)
        mk = (lambda n: Linear(n, ch, ch)) if linear_proj else (lambda n: Conv(n, ch, ch, 1, 1, 0))
        self.proj_in, self.proj_out = mk(f"{name}.proj_in"), mk(f"{name}.proj_out")
        self.blocks = [BasicTransformerBlock(f"{name}.transformer_blocks.{i}", ch, ctx_dim, heads,
                                             sliced) for i in range(layers)]

    def params(self):
        p = {}
        for m in (self.norm, self.proj_in, self.proj_out, *self.blocks):
            p.update(m.params())
        return p

    def __call__(self, W, x, ctx, kv_cache=None):
        h = ops.group_norm(x, W[f"{self.name}.norm.weight"], W[f"{self.name}.norm.bias"],
                           self.groups, 1e-6)
        # proj_in / proj_out are per-pixel linears (1x1 convs in SD1.x): run them
        # on [B, HW, C] tokens, which is a free view in the channels-last layout
        h = _token_linear(W, self.proj_in.name, ops.tokens(h))
        for blk in self.blocks:
            h = blk(W, h, ctx, kv_cache)
        if ops.nhwc():  # channels-last: the residual is a free token view of x
            return ops.untokens(_token_linear(W, self.proj_out.name, h, resid=ops.tokens(x)), x)
        h = _token_linear(W, self.proj_out.name, h)
        return ops.untokens(h, x) + x


def refresh_kv_cache(kv_cache: dict, ctx: torch.Tensor) -> None:
    """Recompute a cross-attention k/v cache IN PLACE for a new text context (the
    tensors may be baked into a captured hipGraph)."""
    for name, kv in kv_cache.items():
        if not name.endswith("@w"):
            w = kv_cache[f"{name}@w"]
            if ops._gemm_ok(ctx, w):
                from ...ops import gemm as G
                G.linear(ctx, w, out=kv)
            else:
                torch.matmul(ctx, w.t(), out=kv)


def _token_linear(W, name, t, resid=None):
    w = W[f"{name}.weight"]
    if w.dim() == 4:
        w = w[:, :, 0, 0]
    return ops.linear(t, w, W.get(f"{name}.bias"), resid=resid)


def timestep_embedding(t: torch.Tensor, dim: int, flip_sin_to_cos: bool, shift: float) -> torch.Tensor:
    half = dim // 2
    exponent = -math.log(10000.0) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - shift)
    emb = t.float()[:, None] * torch.exp(exponent)[None]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], -1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], -1)
    return emb


class UNet2DConditionModel(Module):
    def __init__(self, cfg: UNetConfig):
        self.cfg = cfg
        chans = [b.out_channels for b in cfg.blocks]
        G, eps, ctx, lin, sl = (cfg.norm_num_groups, cfg.norm_eps, cfg.cross_attention_dim,
                                cfg.use_linear_projection, cfg.sliced_attention_size)
        temb = chans[0] * 4
        self.temb_dim = temb
        self.conv_in = Conv("conv_in", cfg.in_channels, chans[0])
        self.t1 = Linear("time_embedding.linear_1", chans[0], temb)
        self.t2 = Linear("time_embedding.linear_2", temb, temb)
        self.down = []
        cout = chans[0]
        for i, b in enumerate(cfg.blocks):
            cin, cout = cout, b.out_channels
            final = i == len(cfg.blocks) - 1
            res, att = [], []
            for j in range(cfg.layers_per_block):
                res.append(ResnetBlock2D(f"down_blocks.{i}.resnets.{j}", cin if j == 0 else cout,
                                         cout, temb, G, eps))
                if b.cross_attn:
                    att.append(Transformer2DModel(f"down_blocks.{i}.attentions.{j}", cout, ctx,
                                                  b.heads, b.transformer_layers, lin, G, sl))
            ds = None if final else Conv(f"down_blocks.{i}.downsamplers.0.conv", cout, cout, 3, 2, 1)
            self.down.append((res, att, ds))
        mid = cfg.blocks[-1]
        cm = chans[-1]
        self.mid_res = [ResnetBlock2D(f"mid_block.resnets.{j}", cm, cm, temb, G, eps) for j in (0, 1)]
        self.mid_att = Transformer2DModel("mid_block.attentions.0", cm, ctx, mid.heads,
                                          mid.transformer_layers, lin, G, sl)
        self.up = []
        rev = list(reversed(chans))
        rblocks = list(reversed(cfg.blocks))
        out_ch = rev[0]
        for i, b in enumerate(rblocks):
            prev_out, out_ch = out_ch, rev[i]
            in_ch = rev[min(i + 1, len(chans) - 1)]
            final = i == len(chans) - 1
            res, att = [], []
            n = cfg.layers_per_block + 1
            for j in range(n):
                skip = in_ch if j == n - 1 else out_ch
                rin = prev_out if j == 0 else out_ch
                res.append(ResnetBlock2D(f"up_blocks.{i}.resnets.{j}", rin + skip, out_ch, temb, G, eps))
                if b.cross_attn:
                    att.append(Transformer2DModel(f"up_blocks.{i}.attentions.{j}", out_ch, ctx,
                                                  b.heads, b.transformer_layers, lin, G, sl))
            us = None if final else Conv(f"up_blocks.{i}.upsamplers.0.conv", out_ch, out_ch)
            self.up.append((res, att, us))
        self.norm_out = Norm("conv_norm_out", chans[0])
        self.conv_out = Conv("conv_out", chans[0], cfg.out_channels)

    def params(self) -> dict[str, tuple]:
        p = {}
        mods = [self.conv_in, self.t1, self.t2, *self.mid_res, self.mid_att, self.norm_out,
                self.conv_out]
        for res, att, s in self.down + self.up:
            mods += res + att + ([s] if s else [])
        for m in mods:
            p.update(m.params())
        return p

    def resnets(self) -> list:
        out = []
        for res, _, _ in self.down:
            out += res
        out += self.mid_res
        for res, _, _ in self.up:
            out += res
        return out

    def _temb_all(self, W):
        """Every ResnetBlock2D's time_emb_proj stacked into ONE weight [sum C, temb]
        (+ bias): the per-step time biases of the whole UNet are one GEMM."""
        key = "@temb_all"
        blocks = [r for r in self.resnets() if r.temb is not None]
        if key not in W:
            W[key] = torch.cat([W[f"{r.temb.name}.weight"] for r in blocks], 0).contiguous()
            W[key + ".bias"] = torch.cat([W[f"{r.temb.name}.bias"] for r in blocks], 0)
        if getattr(self, "_temb_offs", None) is None:
            offs, o = {}, 0
            for r in blocks:
                offs[r.name] = (o, r.temb.cout)
                o += r.temb.cout
            self._temb_offs = offs
        return W[key], W[key + ".bias"], self._temb_offs

    def time_biases(self, W, timestep, B: int, dtype, device, t_index=None) -> dict:
        """{resnet name: time bias [B, C] f32} for this step.

        timestep: a float, a device scalar, or a device table indexed on the device by
        t_index (int32 [1]) — the last two replay unchanged in a hipGraph across steps.
        Device path: sinusoidal-embedding kernel -> linear_1 (+SiLU) -> linear_2 (+SiLU)
        -> one GEMM for every block's time_emb_proj (f32 out)."""
        cfg = self.cfg
        C0 = cfg.blocks[0].out_channels
        wall, ball, offs = self._temb_all(W)
        hip = torch.device(device).type == "cuda" and dtype in (torch.float16, torch.bfloat16)
        if hip:
            from ...ops import gemm as G
            from ...ops import hip as K
            if isinstance(timestep, torch.Tensor):
                tt = timestep.to(device, torch.float32).reshape(-1).contiguous()
            else:
                tt = torch.full((1,), float(timestep), device=device)
            emb = torch.empty(B, C0, device=device, dtype=dtype)
            K.timestep_embed(tt, t_index, B, C0, cfg.flip_sin_to_cos, cfg.freq_shift, emb)
            h = G.linear(emb, W[f"{self.t1.name}.weight"], W[f"{self.t1.name}.bias"], epi="silu")
            st = G.linear(h, W[f"{self.t2.name}.weight"], W[f"{self.t2.name}.bias"], epi="silu")
            tb = torch.empty(B, wall.shape[0], device=device, dtype=torch.float32)
            G.linear(st, wall, ball, epi="store32", resid=tb)
        else:
            if isinstance(timestep, torch.Tensor):
                tv = timestep.reshape(-1)
                tv = tv[int(t_index.item())] if t_index is not None else tv[0]
                t = tv.to(device, torch.float32).expand(B)
            else:
                t = torch.full((B,), float(timestep), device=device)
            emb = timestep_embedding(t, C0, cfg.flip_sin_to_cos, cfg.freq_shift).to(dtype)
            st = F.silu(self.t2(W, F.silu(self.t1(W, emb))))
            tb = F.linear(st, wall, ball).float()
        return {name: tb[:, o:o + c] for name, (o, c) in offs.items()}

    def forward(self, W, sample: torch.Tensor, timestep, ctx: torch.Tensor,
                kv_cache: dict | None = None, t_index=None) -> torch.Tensor:
        """kv_cache: optional dict reused across the steps of ONE generation (fixed ctx);
        holds the cross-attention k/v projections of the context.  timestep: float, device
        scalar, or device table + t_index (see :meth:`time_biases`)."""
        tbs = self.time_biases(W, timestep, sample.shape[0], sample.dtype, sample.device,
                               t_index)
        with ops.layout_nhwc(ops.want_nhwc(sample)):
            # NCHW in and out: conv_in reads the planes, conv_out writes them
            return self._body(W, sample, tbs, ctx, kv_cache)

    # ------------------------------------------------------------------ stages
    # The body as a chain of block-group stages ("down.0" .. "down.{n-1}", "mid",
    # "up.0" .. "up.{n-1}"): the unit of UNet placement across ranks (beyond the
    # reference, which places the UNet whole: sd.rs:200-300).  The state between
    # stages is the running feature map plus the skip stack of the down path.
    def stage_names(self) -> list[str]:
        n = len(self.down)
        return [f"down.{i}" for i in range(n)] + ["mid"] + [f"up.{i}" for i in range(n)]

    def run_stage(self, W, name: str, x: torch.Tensor, skips: list, tbs, ctx, kv_cache):
        """One stage over (x, skips) in the active layout; returns the new (x, skips).
        down.0 takes the NCHW UNet input (conv_in reads it in place); the last up stage
        ends in conv_out, which writes the NCHW UNet output."""
        cfg = self.cfg
        kind, _, idx = name.partition(".")
        if kind == "down":
            i = int(idx)
            if i == 0:
                x = self.conv_in(W, x, in_nchw=True)
                skips = [x]
            res, att, ds = self.down[i]
            for j, r in enumerate(res):
                x = r(W, x, tb=tbs[r.name])
                if att:
                    x = att[j](W, x, ctx, kv_cache)
                skips.append(x)
            if ds is not None:
                x = ds(W, x)
                skips.append(x)
            return x, skips
        if kind == "mid":
            x = self.mid_res[0](W, x, tb=tbs[self.mid_res[0].name])
            x = self.mid_att(W, x, ctx, kv_cache)
            x = self.mid_res[1](W, x, tb=tbs[self.mid_res[1].name])
            return x, skips
        i = int(idx)
        res, att, us = self.up[i]
        for j, r in enumerate(res):
            x = r(W, x, tb=tbs[r.name], skip=skips.pop())
            if att:
                x = att[j](W, x, ctx, kv_cache)
        if us is not None:
            x = us(W, x, up=True)  # nearest-2x upsample fused into the conv
        if i == len(self.up) - 1:
            x = ops.group_norm(x, W["conv_norm_out.weight"], W["conv_norm_out.bias"],
                               cfg.norm_num_groups, cfg.norm_eps, silu=True)
            x = self.conv_out(W, x, out_nchw=True)
        return x, skips

    def forward_stages(self, W, names: list[str], x: torch.Tensor, skips: list, timestep, ctx,
                       kv_cache: dict | None = None, t_index=None):
        """Run consecutive stages: the building block of a UNet split over ranks.  The
        UNet input (before down.0) and output (after the last up stage) are NCHW;
        the (x, skips) handed between stages stay in the active internal layout (the
        ranks of one job share it), so a hop moves them as they are."""
        B = x.shape[0]
        tbs = self.time_biases(W, timestep, B, x.dtype, x.device, t_index)
        # (down.0 reads / the last up stage writes the NCHW layout itself)
        with ops.layout_nhwc(ops.want_nhwc(x)):
            for n in names:
                x, skips = self.run_stage(W, n, x, skips, tbs, ctx, kv_cache)
            return x, skips

    def _body(self, W, sample, tbs, ctx, kv_cache):
        x, skips = sample, []
        for n in self.stage_names():
            x, skips = self.run_stage(W, n, x, skips, tbs, ctx, kv_cache)
        return x
