"""Native Stable Diffusion engine (csrc/engine/sd_engine.cpp via cake_amd/sd_engine.py)
against the Python pipeline on the same synthetic checkpoint (the mini architecture:
every shape on the HIP kernels), convolution autotuning off on both sides (the static
planner: the same variants):

  * each component — text encoder(s), one UNet forward, the VAE decode — agrees with
    the Python module to f16 rounding;
  * a whole guided generation (DDIM for v1-5 and, with v-prediction, v2-1 /
    Euler-ancestral for turbo, graph replays
    after the first step) ends in the same latents as SDUnit.denoise and the same image.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DT = torch.float16


@pytest.fixture(scope="module", params=["v1-5", "v2-1", "xl", "turbo"])
def mini(request, tmp_path_factory):
    from cake_amd.models.sd.config import mini_config
    from cake_amd.models.sd.weights import write_sd_checkpoint
    v = request.param
    d = tmp_path_factory.mktemp(f"sd_mini_{v}")
    cfg = mini_config(v)
    write_sd_checkpoint(d, cfg, torch.float16, seed=5, mini=True)
    return v, cfg, d


@pytest.fixture(autouse=True)
def _static_conv_plans(monkeypatch):
    import cake_amd.ops.conv as conv
    monkeypatch.setattr(conv, "_AUTOTUNE", False)
    conv._cache.clear()


def _engine(d):
    from cake_amd.sd_engine import NativeSD
    return NativeSD(str(d), dtype="f16", autotune=False)


def _weights(name, cfg, d, version):
    from cake_amd.models.sd.weights import load_component, resolve
    return load_component(name, resolve(name, None, version, True, d), cfg, "cuda:0", DT)


def _ids(seed, vocab):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, vocab - 2, (77,), generator=g)
    ids[0] = vocab - 2
    ids[20:] = vocab - 1
    return ids.to(torch.int32)


def _close(a, b, tol):
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    err = float(np.max(np.abs(a - b)))
    scale = float(np.max(np.abs(b))) + 1e-6
    assert err <= tol * scale, (err, scale)


def test_text_encoders_match_python(cuda, mini):
    from cake_amd.models.sd.clip import ClipTextTransformer
    v, cfg, d = mini
    eng = _engine(d)
    encs = [("clip", cfg.clip)] + ([("clip2", cfg.clip2)] if cfg.clip2 else [])
    for which, (name, ccfg) in enumerate(encs):
        W = _weights(name, cfg, d, v)
        ids = _ids(3 + which, ccfg.vocab_size)
        ref = ClipTextTransformer(ccfg, W).forward(ids[None].cuda()).float().cpu().numpy()
        got = eng.text(which, ids.numpy()[None])
        _close(got, ref, 2e-3)
    eng.close()


def test_unet_forward_matches_python(cuda, mini):
    from cake_amd.models.sd.unet import UNet2DConditionModel
    v, cfg, d = mini
    eng = _engine(d)
    W = _weights("unet", cfg, d, v)
    g = torch.Generator().manual_seed(7)
    h, w = cfg.height // 8, cfg.width // 8
    sample = torch.randn(2, 4, h, w, generator=g)
    ctx = torch.randn(2, 77, cfg.unet.cross_attention_dim, generator=g)
    ref = UNet2DConditionModel(cfg.unet).forward(W, sample.cuda().to(DT), 501.0,
                                                  ctx.cuda().to(DT), kv_cache={})
    # the engine rounds its f32 inputs to the model dtype exactly as .to(DT) does
    got = eng.unet(sample.to(DT).float().numpy(), 501.0, ctx.to(DT).float().numpy())
    _close(got, ref.float().cpu().numpy(), 2e-3)
    eng.close()


def test_vae_decode_matches_python(cuda, mini):
    from cake_amd.models.sd.vae import AutoencoderKL
    v, cfg, d = mini
    eng = _engine(d)
    W = _weights("vae", cfg, d, v)
    g = torch.Generator().manual_seed(9)
    z = torch.randn(1, 4, cfg.height // 8, cfg.width // 8, generator=g).to(DT)
    ref = AutoencoderKL(cfg.vae).decode(W, z.cuda()).float().cpu().numpy()[:, :3]
    got = eng.vae_decode(z.float().numpy())
    _close(got, ref, 2e-3)
    eng.close()


def test_generation_matches_python_denoise(cuda, mini):
    """Whole generation: text -> guided steps (graph replays) -> VAE, against the Python
    components driven the way SDGenerator drives them."""
    from cake_amd.models.sd.clip import ClipTextTransformer
    from cake_amd.models.sd.schedulers import build_scheduler
    from cake_amd.models.sd.shardable import SDUnit
    from cake_amd.models.sd.vae import AutoencoderKL
    from cake_amd.ops import hip as K
    v, cfg, d = mini
    steps = 4 if v != "turbo" else 2
    guidance = 7.5 if v != "turbo" else 2.0
    seed = 1234567
    encs = [("clip", cfg.clip)] + ([("clip2", cfg.clip2)] if cfg.clip2 else [])
    ids = {}
    embs = []
    for k, (name, ccfg) in enumerate(encs):
        cond, unc = _ids(11 + k, ccfg.vocab_size), _ids(21 + k, ccfg.vocab_size)
        ids[k] = (cond, unc)
        m = ClipTextTransformer(ccfg, _weights(name, cfg, d, v))
        e = m.forward(cond[None].cuda())
        u = m.forward(unc[None].cuda())
        embs.append(torch.cat([u, e], 0))
    emb = torch.cat(embs, -1)
    sched = build_scheduler(cfg.scheduler, steps)
    g = torch.Generator().manual_seed(5)
    noise = torch.randn(1, 4, cfg.height // 8, cfg.width // 8, generator=g)
    latents = (noise.cuda() * sched.init_noise_sigma).float()
    unit = SDUnit("unet", cfg, _weights("unet", cfg, d, v), torch.device("cuda:0"), DT)
    ref_x, _ = unit.denoise(latents, emb, sched, sched.timesteps(), guidance, True, seed)
    vae = AutoencoderKL(cfg.vae)
    img = vae.decode(_weights("vae", cfg, d, v), (ref_x / cfg.vae_scale).to(DT))
    ref_rgb = K.to_rgb8(img[:, :3].contiguous()).cpu().numpy()[0]

    eng = _engine(d)
    kw = dict(cond=ids[0][0].numpy(), uncond=ids[0][1].numpy())
    if cfg.clip2 is not None:
        kw.update(cond2=ids[1][0].numpy(), uncond2=ids[1][1].numpy())
    out = eng.generate(n_steps=steps, guidance=guidance, seed=seed, init_noise=noise.numpy(), **kw)
    _close(out.latents, ref_x.cpu().numpy()[0], 2e-3)
    diff = np.abs(out.rgb.astype(np.int32) - ref_rgb.astype(np.int32))
    assert diff.mean() < 0.5 and diff.max() <= 8, (diff.mean(), diff.max())
    assert len(out.step_s) == steps and all(s > 0 for s in out.step_s)
    # a second generation on the same engine replays the captured step
    again = eng.generate(n_steps=steps, guidance=guidance, seed=seed, init_noise=noise.numpy(),
                         **kw)
    assert np.array_equal(again.rgb, out.rgb) and np.array_equal(again.latents, out.latents)
    # eager steps give the same latents as the replays
    eager = eng.generate(n_steps=steps, guidance=guidance, seed=seed, init_noise=noise.numpy(),
                         use_graph=False, **kw)
    assert np.array_equal(eager.latents, out.latents)
    eng.close()


def test_master_serves_images_from_the_native_engine(cuda, mini, tmp_path, monkeypatch):
    """The CLI / API master picks the native engine for an all-local model; the same seed
    and prompt give the same image as the Python pipeline (CAKE_NATIVE=0)."""
    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import _load_image
    from cake_amd.models.sd.args import ImageGenerationArgs
    from cake_amd.models.sd.native_generator import NativeSDGenerator
    v, cfg, d = mini
    topo = tmp_path / "empty.yml"
    topo.write_text("{}\n")
    args = build_parser().parse_args(["--model", str(d), "--topology", str(topo), "--model-type",
                                      "image-model", "--sd-version", v, "--dtype", "f16"])
    ctx = Context.from_args(args)
    monkeypatch.setenv("CAKE_CONV_AUTOTUNE", "0")
    native = _load_image(ctx)
    assert isinstance(native, NativeSDGenerator)
    native.eng.close()
    native.eng = __import__("cake_amd.sd_engine", fromlist=["NativeSD"]).NativeSD(
        str(d), dtype="f16", autotune=False)  # static conv plans, as the Python side below
    req = ImageGenerationArgs(image_prompt="a red cube", uncond_prompt="blurry", n_steps=3,
                              image_seed=42)
    got = []
    native.generate_image(req, lambda imgs: got.append(imgs))
    monkeypatch.setenv("CAKE_NATIVE", "0")
    py = _load_image(ctx)
    assert not isinstance(py, NativeSDGenerator)
    ref = []
    py.generate_image(req, lambda imgs: ref.append(imgs))
    a = np.asarray(got[-1][0], dtype=np.int32)
    b = np.asarray(ref[-1][0], dtype=np.int32)
    assert a.shape == b.shape == (cfg.height, cfg.width, 3)
    assert np.abs(a - b).mean() < 0.5 and np.abs(a - b).max() <= 8
    assert len(native.last_step_s) == 3


def test_native_sd_tcp_worker_serves_the_unet(cuda, mini, tmp_path, monkeypatch):
    """cake-cli --mode worker on an image model serves its topology components (here the
    UNet and the VAE, encode and decode) from the native SD engine — the reference's packed-tensor SingleOp interface,
    no interpreter in the worker; the Python master's image over it matches its all-local
    image (the master's host-side scheduler math vs the fused kernel: a few grey levels)."""
    import os
    import socket
    import subprocess
    import time

    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import _load_image
    from cake_amd.models.sd.args import ImageGenerationArgs
    v, cfg, d = mini
    if v != "v1-5":
        pytest.skip("one version covers the worker plumbing")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{port}'\n  layers:\n    - 'unet'\n    - 'vae'\n")
    empty = tmp_path / "empty.yml"
    empty.write_text("{}\n")
    env = dict(os.environ, CAKE_LOG="warning")
    w = subprocess.Popen([cli, "--mode", "worker", "--name", "w1", "--model", str(d),
                          "--topology", str(topo), "--address", f"127.0.0.1:{port}",
                          "--model-type", "image-model", "--sd-version", v, "--dtype", "f16"],
                         cwd=root, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                         text=True)
    monkeypatch.setenv("CAKE_NATIVE", "0")  # the master: the Python pipeline both times
    req = ImageGenerationArgs(image_prompt="a red cube", uncond_prompt="", n_steps=3,
                              image_seed=3)
    try:
        t0 = time.time()
        while True:
            if w.poll() is not None:
                raise AssertionError(f"worker exited: {w.stderr.read()[-3000:]}")
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
                break
            except OSError:
                assert time.time() - t0 < 180, "worker did not listen"
                time.sleep(0.3)

        def image(topology, r=req):
            args = build_parser().parse_args(["--model", str(d), "--topology", str(topology),
                                              "--model-type", "image-model", "--sd-version", v,
                                              "--dtype", "f16"])
            gen = _load_image(Context.from_args(args))
            out = []
            gen.generate_image(r, lambda imgs: out.append(imgs))
            return out[-1][0]
        remote_img = image(topo)
        remote = np.asarray(remote_img, dtype=np.int32)
        local = np.asarray(image(empty), dtype=np.int32)
        # img2img through the worker's VAE encoder (its own posterior normals: shape only)
        src = tmp_path / "src.png"
        remote_img.save(src)
        i2i = image(topo, ImageGenerationArgs(image_prompt="a red cube", n_steps=4,
                                              img2img=str(src), img2img_strength=0.5,
                                              image_seed=4))
        assert i2i.size == (cfg.width, cfg.height)
    finally:
        w.kill()
        err = w.communicate()[1]
    assert "native SD worker" in err, err[-2000:]
    assert remote.shape == local.shape
    diff = np.abs(remote - local)
    assert diff.mean() < 2.0 and diff.max() <= 32, (diff.mean(), diff.max())


@pytest.mark.parametrize("bsize", [1, 2])
def test_img2img_on_the_native_engine_matches_python(cuda, mini, tmp_path, monkeypatch, bsize):
    """img2img natively (the engine's VAE encoder, the pipeline's sampling and noise draws,
    the denoise from t_start) gives the Python pipeline's image; at bsize 2 both images
    start from the encoded image with their own noise."""
    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import _load_image
    from cake_amd.models.sd.args import ImageGenerationArgs
    from cake_amd.models.sd.native_generator import NativeSDGenerator
    from cake_amd.sd_engine import NativeSD
    v, cfg, d = mini
    topo = tmp_path / "empty.yml"
    topo.write_text("{}\n")
    args = build_parser().parse_args(["--model", str(d), "--topology", str(topo), "--model-type",
                                      "image-model", "--sd-version", v, "--dtype", "f16"])
    ctx = Context.from_args(args)
    native = _load_image(ctx)
    assert isinstance(native, NativeSDGenerator)
    native.eng.close()
    native.eng = NativeSD(str(d), dtype="f16", autotune=False)
    src = []
    native.generate_image(ImageGenerationArgs(image_prompt="a blue sphere", n_steps=2,
                                              image_seed=1), lambda imgs: src.append(imgs))
    path = tmp_path / "src.png"
    src[-1][0].save(path)
    req = ImageGenerationArgs(image_prompt="a red cube", n_steps=4, img2img=str(path),
                              img2img_strength=0.5, image_seed=8, bsize=bsize)
    got = []
    native.generate_image(req, lambda imgs: got.append(imgs))
    assert native._fallback is None  # served natively
    assert len(native.last_step_s) == 2  # t_start = 4 - int(4 * 0.5)
    monkeypatch.setenv("CAKE_NATIVE", "0")
    py = _load_image(ctx)
    ref = []
    py.generate_image(req, lambda imgs: ref.append(imgs))
    assert len(got[-1]) == len(ref[-1]) == bsize
    for k in range(bsize):
        a = np.asarray(got[-1][k], dtype=np.int32)
        b = np.asarray(ref[-1][k], dtype=np.int32)
        assert np.abs(a - b).mean() < 0.5 and np.abs(a - b).max() <= 8, (
            k, np.abs(a - b).mean(), np.abs(a - b).max())
    if bsize > 1:  # distinct noise per image
        assert np.abs(np.asarray(got[-1][0], np.int32) - np.asarray(got[-1][1], np.int32)).max() > 0


def test_bsize_and_intermediary_images_on_the_native_engine(cuda, mini, tmp_path, monkeypatch):
    """bsize 2 (the UNet over 4 rows with the reference's repeated text rows) and an
    intermediary image every second step, natively: the same callbacks (count, image
    count per call) and images as the Python pipeline."""
    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import _load_image
    from cake_amd.models.sd.args import ImageGenerationArgs
    from cake_amd.models.sd.native_generator import NativeSDGenerator
    from cake_amd.sd_engine import NativeSD
    v, cfg, d = mini
    topo = tmp_path / "empty.yml"
    topo.write_text("{}\n")
    args = build_parser().parse_args(["--model", str(d), "--topology", str(topo), "--model-type",
                                      "image-model", "--sd-version", v, "--dtype", "f16"])
    ctx = Context.from_args(args)
    native = _load_image(ctx)
    assert isinstance(native, NativeSDGenerator)
    native.eng.close()
    native.eng = NativeSD(str(d), dtype="f16", autotune=False)
    req = ImageGenerationArgs(image_prompt="a red cube", uncond_prompt="blurry", n_steps=4,
                              image_seed=5, bsize=2, intermediary_images=2)
    got = []
    native.generate_image(req, lambda imgs: got.append(imgs))
    assert native._fallback is None  # served natively
    assert len(native.last_step_s) == 4
    monkeypatch.setenv("CAKE_NATIVE", "0")
    py = _load_image(ctx)
    ref = []
    py.generate_image(req, lambda imgs: ref.append(imgs))
    # steps 0 and 2 (i % 2 == 0), then the final images
    assert len(got) == len(ref) == 3 and all(len(x) == 2 for x in got + ref)
    for g, r in zip(got, ref):
        for gi, ri in zip(g, r):
            a, b = np.asarray(gi, dtype=np.int32), np.asarray(ri, dtype=np.int32)
            assert a.shape == b.shape == (cfg.height, cfg.width, 3)
            assert np.abs(a - b).mean() < 0.5 and np.abs(a - b).max() <= 8, (
                np.abs(a - b).mean(), np.abs(a - b).max())


def test_native_engine_writes_the_chrome_trace(cuda, mini, tmp_path, monkeypatch):
    """--sd-tracing on the native engine: a Chrome trace with the pipeline's spans (text
    embeddings, one per step, VAE decode) from the engine's timings, no Python fallback."""
    import json

    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import _load_image
    from cake_amd.models.sd.args import ImageGenerationArgs
    from cake_amd.models.sd.native_generator import NativeSDGenerator
    v, cfg, d = mini
    if v != "v1-5":
        pytest.skip("one version covers the trace plumbing")
    topo = tmp_path / "empty.yml"
    topo.write_text("{}\n")
    args = build_parser().parse_args(["--model", str(d), "--topology", str(topo), "--model-type",
                                      "image-model", "--sd-version", v, "--dtype", "f16"])
    native = _load_image(Context.from_args(args))
    assert isinstance(native, NativeSDGenerator)
    monkeypatch.chdir(tmp_path)
    got = []
    native.generate_image(ImageGenerationArgs(image_prompt="a red cube", n_steps=3, image_seed=2,
                                              tracing=True), lambda imgs: got.append(imgs))
    assert native._fallback is None and len(got) == 1
    traces = list(tmp_path.glob("trace-*.json"))
    assert len(traces) == 1
    names = [e["name"] for e in json.loads(traces[0].read_text())["traceEvents"]]
    assert "text_embeddings" in names and "vae_decode" in names
    assert [n for n in names if n.startswith("step ")] == ["step 1", "step 2", "step 3"]
    native.eng.close()


@pytest.mark.parametrize("served", [("unet", "vae"), ("clip", "unet", "vae")])
def test_native_master_with_remote_sd_components(cuda, mini, tmp_path, monkeypatch, served):
    """The native SD engine as the master of an image topology: the UNet and the VAE on a
    TCP worker (cake-cli --mode worker, the native SD worker), the text encoders local —
    every step one SingleOp round trip through the engine's own client.  The image equals
    the all-local native image (the same kernels; the worker's f32 wire round trip and the
    host-side RGB8 conversion: a grey level)."""
    import os
    import socket
    import subprocess
    import time

    from cake_amd.cli import build_parser
    from cake_amd.context import Context
    from cake_amd.master import _load_image
    from cake_amd.models.sd.args import ImageGenerationArgs
    from cake_amd.models.sd.native_generator import NativeSDGenerator
    v, cfg, d = mini
    if v != "v1-5":
        pytest.skip("one version covers the remote plumbing")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{port}'\n  layers:\n" +
                    "".join(f"    - '{c}'\n" for c in served))
    empty = tmp_path / "empty.yml"
    empty.write_text("{}\n")
    env = dict(os.environ, CAKE_LOG="warning")
    w = subprocess.Popen([cli, "--mode", "worker", "--name", "w1", "--model", str(d),
                          "--topology", str(topo), "--address", f"127.0.0.1:{port}",
                          "--model-type", "image-model", "--sd-version", v, "--dtype", "f16"],
                         cwd=root, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                         text=True)
    req = ImageGenerationArgs(image_prompt="a red cube", uncond_prompt="blurry", n_steps=3,
                              image_seed=7)
    gens = []
    try:
        t0 = time.time()
        while True:
            if w.poll() is not None:
                raise AssertionError(f"worker exited: {w.stderr.read()[-3000:]}")
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
                break
            except OSError:
                assert time.time() - t0 < 180, "worker did not listen"
                time.sleep(0.3)

        def image(topology):
            args = build_parser().parse_args(["--model", str(d), "--topology", str(topology),
                                              "--model-type", "image-model", "--sd-version", v,
                                              "--dtype", "f16"])
            gen = _load_image(Context.from_args(args))
            gens.append(gen)
            out = []
            gen.generate_image(req, lambda imgs: out.append(imgs))
            return gen, out[-1][0]
        rg, remote_img = image(topo)
        assert isinstance(rg, NativeSDGenerator) and rg._fallback is None
        assert sorted(rg.eng.remote) == sorted(served)
        assert len(rg.last_step_s) == 3
        lg, local_img = image(empty)
        assert isinstance(lg, NativeSDGenerator) and not lg.eng.remote
        if "vae" in served:  # img2img through the worker's VAE, natively
            import torch

            from cake_amd.models.sd.pipeline import image_preprocess
            init = tmp_path / "init.png"
            remote_img.save(init)
            smp = rg._encode_image(str(init)).float().cpu()  # the worker's posterior sample
            mo = torch.from_numpy(lg.eng.vae_encode(image_preprocess(str(init)).numpy()))
            mean, logvar = mo.chunk(2, 1)
            z = (smp - mean) / torch.exp(0.5 * logvar.clamp(-30.0, 20.0))
            assert torch.isfinite(z).all() and z.abs().max() < 8, z.abs().max()
            assert 0.7 < float(z.std()) < 1.3, float(z.std())   # mean + std * N(0, 1)
            out2 = []
            rg.generate_image(ImageGenerationArgs(image_prompt="a red cube", n_steps=4,
                                                  image_seed=3, img2img=str(init),
                                                  img2img_strength=0.5),
                              lambda imgs: out2.append(imgs))
            assert rg._fallback is None and len(rg.last_step_s) == 2
            assert np.asarray(out2[-1][0]).shape == (cfg.height, cfg.width, 3)
    finally:
        for g in gens:
            g.eng.close()
        w.kill()
        err = w.communicate()[1]
    assert "native SD worker" in err, err[-2000:]
    a = np.asarray(remote_img, dtype=np.int32)
    b = np.asarray(local_img, dtype=np.int32)
    assert a.shape == b.shape == (cfg.height, cfg.width, 3)
    diff = np.abs(a - b)
    assert diff.mean() < 0.5 and diff.max() <= 2, (diff.mean(), diff.max())


def test_native_sd_master_fails_loudly_when_the_unet_worker_dies(cuda, mini, tmp_path):
    """Failure detection on the native SD engine's TCP client: a generation through a live
    UNet worker succeeds; after the worker is killed the next one raises (connection error
    or the remote timeout) instead of hanging or returning an image."""
    import os
    import socket
    import subprocess
    import time

    from cake_amd.sd_engine import NativeSD
    v, cfg, d = mini
    if v != "v1-5":
        pytest.skip("one version covers the client's failure path")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cli = os.path.join(root, "cake_amd", "lib", "cake-cli")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    topo = tmp_path / "topology.yml"
    topo.write_text(f"w1:\n  host: '127.0.0.1:{port}'\n  layers:\n    - 'unet'\n")
    w = subprocess.Popen([cli, "--mode", "worker", "--name", "w1", "--model", str(d),
                          "--topology", str(topo), "--address", f"127.0.0.1:{port}",
                          "--model-type", "image-model", "--sd-version", v, "--dtype", "f16"],
                         cwd=root, env=dict(os.environ, CAKE_LOG="warning"),
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    eng = None
    try:
        t0 = time.time()
        while True:
            if w.poll() is not None:
                raise AssertionError(f"worker exited: {w.stderr.read()[-3000:]}")
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
                break
            except OSError:
                assert time.time() - t0 < 180, "worker did not listen"
                time.sleep(0.3)
        eng = NativeSD(str(d), dtype="f16", autotune=False, remote={"unet": f"127.0.0.1:{port}"},
                       remote_timeout_s=10.0)
        ids = _ids(1, cfg.clip.vocab_size).numpy()
        out = eng.generate(ids, ids, n_steps=2, guidance=7.5, seed=1)
        assert out.rgb.shape[-1] == 3 and len(out.step_s) == 2
        w.kill()
        w.wait(timeout=30)
        t0 = time.time()
        with pytest.raises(RuntimeError):
            eng.generate(ids, ids, n_steps=2, guidance=7.5, seed=1)
        assert time.time() - t0 < 60
    finally:
        if eng is not None:
            eng.close()
        if w.poll() is None:
            w.kill()
        w.communicate()
