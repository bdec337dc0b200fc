"""Stable Diffusion pipeline on CPU (tiny structurally-complete configs, f32).

Covers every version's block layout, CFG, img2img, intermediary images, bsize,
the packing codec, schedulers, and component placement on a TCP worker
(identical images local vs remote)."""
import json

import pytest
import torch

from cake_amd.cli import build_parser
from cake_amd.context import Context
from cake_amd.models.sd.args import ImageGenerationArgs
from cake_amd.models.sd.config import SchedulerConfig, get_config, tiny_config
from cake_amd.models.sd.pipeline import SDGenerator
from cake_amd.models.sd.schedulers import build_scheduler
from cake_amd.models.sd.util import pack_tensors, unpack_tensors
from cake_amd.models.sd.weights import component_shapes, write_sd_checkpoint


def _ctx(d, topo, *extra):
    args = build_parser().parse_args(["--model", str(d), "--topology", str(topo), "--cpu",
                                      "--model-type", "image-model", *extra])
    return Context.from_args(args)


@pytest.fixture(scope="module", params=["v1-5", "v2-1", "xl", "turbo"])
def sd_dir(request, tmp_path_factory):
    d = tmp_path_factory.mktemp(f"sd-{request.param}")
    write_sd_checkpoint(d, tiny_config(request.param), torch.float32, tiny=True)
    (d / "empty.yml").write_text("{}\n")
    return request.param, d


def test_generate_local(sd_dir, tmp_path):
    version, d = sd_dir
    gen = SDGenerator.load(_ctx(d, d / "empty.yml", "--sd-version", version))
    got = []
    args = ImageGenerationArgs(image_prompt="a cat", n_steps=3, bsize=2, image_seed=7,
                               intermediary_images=2)
    gen.generate_image(args, lambda imgs: got.append(imgs))
    assert len(got) == 3 and all(len(b) == 2 for b in got)  # steps 0 and 2 + final
    assert got[-1][0].size == (64, 64) and got[-1][0].mode == "RGB"
    # determinism with a seed
    again = []
    gen.generate_image(args, lambda imgs: again.append(imgs))
    assert again[-1][0].tobytes() == got[-1][0].tobytes()
    # img2img
    src = tmp_path / "in.png"
    got[-1][0].save(src)
    out = []
    gen.generate_image(ImageGenerationArgs(n_steps=4, img2img=str(src), img2img_strength=0.5,
                                           image_seed=1), lambda imgs: out.append(imgs))
    assert out and out[-1][0].size == (64, 64)
    # img2img at bsize 2: both images from the encoded image, each with its own noise
    out2 = []
    gen.generate_image(ImageGenerationArgs(n_steps=4, img2img=str(src), img2img_strength=0.5,
                                           image_seed=1, bsize=2), lambda imgs: out2.append(imgs))
    assert len(out2[-1]) == 2 and all(im.size == (64, 64) for im in out2[-1])


def test_unet_on_worker_matches_local(tmp_path):
    from cake_amd.parallel.worker import Worker
    d = tmp_path / "sd"
    write_sd_checkpoint(d, tiny_config("v1-5"), torch.float32, tiny=True)
    (d / "empty.yml").write_text("{}\n")
    wt = d / "w.yml"
    wt.write_text("gpu1:\n  host: '127.0.0.1:0'\n  layers: [unet, vae]\n")
    w = Worker(_ctx(d, wt, "--mode", "worker", "--name", "gpu1", "--address", "127.0.0.1:0"))
    w.serve_in_thread()
    try:
        topo = d / "t.yml"
        topo.write_text(f"gpu1:\n  host: '127.0.0.1:{w.port}'\n  layers:\n    - unet\n    - vae\n")
        args = ImageGenerationArgs(image_prompt="x", n_steps=2, image_seed=3)
        imgs = {}
        for name, t in (("local", d / "empty.yml"), ("remote", topo)):
            gen = SDGenerator.load(_ctx(d, t))
            res = []
            gen.generate_image(args, lambda i: res.append(i))
            imgs[name] = res[-1][0].tobytes()
        assert imgs["local"] == imgs["remote"]
    finally:
        w.stop()


def test_pack_unpack_layout():
    a, b = torch.randn(2, 3), torch.tensor([5.0])
    p = pack_tensors([a, b])
    assert p[:4].tolist() == [2.0, 2.0, 2.0, 3.0]
    ua, ub = unpack_tensors(p)
    assert torch.equal(ua, a) and torch.equal(ub, b)


def test_schedulers():
    ddim = build_scheduler(SchedulerConfig(), 30)
    assert ddim.timesteps()[0] == 30 * 33 - 33 + 1 and ddim.timesteps()[-1] == 1
    x = torch.randn(1, 4, 8, 8)
    # x0-consistency: a perfect epsilon prediction recovers the clean sample at the end
    x0 = torch.randn(1, 4, 8, 8)
    eps = torch.randn(1, 4, 8, 8)
    t = ddim.timesteps()[-1]
    xt = ddim.add_noise(x0, eps, t)
    a_prev = float(ddim.acp[0])  # final step: prev timestep < 0 -> alphas_cumprod[0]
    expect = a_prev ** 0.5 * x0 + (1 - a_prev) ** 0.5 * eps
    assert torch.allclose(ddim.step(eps, t, xt), expect, atol=1e-4)
    ea = build_scheduler(SchedulerConfig(kind="euler_ancestral", timestep_spacing="trailing"), 1)
    assert ea.timesteps() == [999] and ea.init_noise_sigma > 10
    assert torch.isfinite(ea.step(torch.zeros_like(x), 999, x)).all()


def test_full_size_configs_match_known_parameter_counts():
    """Architectures match the diffusers checkpoints exactly (SDXL without the
    add_embedding / text_projection that cake does not use)."""
    n = lambda shapes: sum(int(torch.tensor(s).prod()) for s in shapes.values())
    v15, v21, xl = get_config("v1-5"), get_config("v2-1"), get_config("xl")
    assert n(component_shapes("unet", v15)) == 859520964
    assert n(component_shapes("vae", v15)) == 83653863
    assert n(component_shapes("clip", v15)) == 123060480
    assert n(component_shapes("unet", v21)) == 865910724
    assert n(component_shapes("clip", v21)) == 340387840
    assert n(component_shapes("unet", xl)) == 2567463684 - 5245440
    assert n(component_shapes("clip2", xl)) == 694659840 - 1280 * 1280
