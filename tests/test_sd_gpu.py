"""SD components on the GPU kernel path vs the PyTorch CPU reference (tiny configs)."""
import pytest
import torch

from cake_amd.models.sd.config import tiny_config
from cake_amd.models.sd.clip import ClipTextTransformer
from cake_amd.models.sd.unet import UNet2DConditionModel
from cake_amd.models.sd.vae import AutoencoderKL
from cake_amd.models.sd.weights import random_component

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("version", ["v1-5", "xl"])
def test_unet_vae_clip_gpu_vs_cpu(cuda, version):
    cfg = tiny_config(version)
    dt = torch.float16
    wu = random_component("unet", cfg, "cpu", torch.float32)
    unet = UNet2DConditionModel(cfg.unet)
    x = torch.randn(2, 4, 8, 8)
    ctx = torch.randn(2, 77, cfg.unet.cross_attention_dim)
    ref = unet.forward(wu, x, 500, ctx)
    gw = {k: v.to(cuda, dt) for k, v in wu.items()}
    out = unet.forward(gw, x.to(cuda, dt), 500, ctx.to(cuda, dt))
    torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=3e-2)

    wv = random_component("vae", cfg, "cpu", torch.float32)
    vae = AutoencoderKL(cfg.vae)
    z = torch.randn(1, 4, 8, 8)
    ref = vae.decode(wv, z)
    out = vae.decode({k: v.to(cuda, dt) for k, v in wv.items()}, z.to(cuda, dt))
    torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=3e-2)

    wc = random_component("clip", cfg, "cpu", torch.float32)
    ids = torch.randint(0, cfg.clip.vocab_size, (1, 77))
    ref = ClipTextTransformer(cfg.clip, wc).forward(ids)
    out = ClipTextTransformer(cfg.clip, {k: v.to(cuda, dt) for k, v in wc.items()}).forward(ids.to(cuda))
    torch.testing.assert_close(out.float().cpu(), ref, atol=3e-2, rtol=3e-2)


def test_unet_vae_channels_last_kernels_gpu_vs_cpu(cuda):
    """Channel widths that are multiples of 64, so every conv runs the MFMA
    implicit-GEMM kernels (im2col, halo, fused upsample, split-K) and GroupNorm
    the channels-last kernel; checked against the NCHW f32 CPU reference."""
    import dataclasses
    from cake_amd.models.sd.config import UNetBlock
    base = tiny_config("v1-5")
    unet_cfg = dataclasses.replace(base.unet, blocks=[UNetBlock(64, True, 2), UNetBlock(128, True, 4),
                                                      UNetBlock(128, False, 4)],
                                   cross_attention_dim=64, norm_num_groups=8)
    vae_cfg = dataclasses.replace(base.vae, block_out_channels=(64, 64, 128, 128))
    cfg = dataclasses.replace(base, unet=unet_cfg, vae=vae_cfg)
    dt = torch.bfloat16
    wu = random_component("unet", cfg, "cpu", torch.float32)
    unet = UNet2DConditionModel(cfg.unet)
    x = torch.randn(2, 4, 16, 16)
    ctx = torch.randn(2, 77, 64)
    ref = unet.forward(wu, x, 500, ctx)
    gw = {k: v.to(cuda, dt) for k, v in wu.items()}
    out = unet.forward(gw, x.to(cuda, dt), 500, ctx.to(cuda, dt))
    assert any(k.endswith("@nhwc") for k in gw), "channels-last conv path not taken"
    torch.testing.assert_close(out.float().cpu(), ref, atol=6e-2, rtol=6e-2)

    wv = random_component("vae", cfg, "cpu", torch.float32)
    vae = AutoencoderKL(cfg.vae)
    z = torch.randn(1, 4, 8, 8)
    ref = vae.decode(wv, z)
    out = vae.decode({k: v.to(cuda, dt) for k, v in wv.items()}, z.to(cuda, dt))
    torch.testing.assert_close(out.float().cpu(), ref, atol=6e-2, rtol=6e-2)
    img = torch.rand(1, 3, 64, 64) * 2 - 1
    g = torch.Generator().manual_seed(0)
    ref = vae.encode(wv, img, g)
    g = torch.Generator().manual_seed(0)
    out = vae.encode({k: v.to(cuda, dt) for k, v in wv.items()}, img.to(cuda, dt), g)
    torch.testing.assert_close(out.float().cpu(), ref, atol=6e-2, rtol=6e-2)


def test_unet_unit_graph_replay_matches_eager(cuda):
    """SDUnit replays the UNet step as a hipGraph; a new text embedding refreshes the
    cached cross-attention k/v in place; outputs equal the eager forward."""
    import dataclasses
    from cake_amd.models.sd.config import UNetBlock
    from cake_amd.models.sd.shardable import SDUnit
    from cake_amd.models.sd.util import pack_tensors
    base = tiny_config("v1-5")
    ucfg = dataclasses.replace(base.unet, blocks=[UNetBlock(64, True, 2), UNetBlock(128, False, 4)],
                               cross_attention_dim=64, norm_num_groups=8)
    cfg = dataclasses.replace(base, unet=ucfg)
    dt = torch.bfloat16
    w = {k: v.to(cuda, dt) for k, v in random_component("unet", cfg, "cpu", torch.float32).items()}
    unit = SDUnit("unet", cfg, w, cuda, dt)
    assert unit.use_graph
    lat = torch.randn(2, 4, 16, 16, device=cuda).to(dt)
    e1 = torch.randn(2, 77, 64, device=cuda).to(dt)
    e2 = torch.randn(2, 77, 64, device=cuda).to(dt)
    eager = UNet2DConditionModel(cfg.unet)
    for emb, t in ((e1, 500.0), (e1, 300.0), (e2, 500.0), (e1, 100.0)):
        got = unit.forward(pack_tensors([lat, emb, torch.tensor([t], device=cuda)], cuda))
        with torch.no_grad():
            ref = eager.forward(w, lat, t, emb)
        torch.testing.assert_close(got.float(), ref.float(), atol=3e-2, rtol=3e-2)
    assert len(unit._graphs) == 1
