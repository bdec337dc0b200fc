"""The native engine's split UNet (csrc/engine/sd_engine.cpp, CakeSdSplitOpts; BASELINE
config 5): the UNet's stages over 2 and 3 ranks sharing one GPU, every step one graph
replay per rank with device bulk hops (feature map run to run, each skip once from its
producer to its consumer, the prediction back to rank 0), gives the single-rank engine's
latents and image bit for bit (the same kernels on the same data in the same order)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ids(seed, vocab):
    r = np.random.default_rng(seed)
    ids = r.integers(0, vocab - 2, 77).astype(np.int32)
    ids[0] = vocab - 2
    ids[20:] = vocab - 1
    return ids


GEN = dict(n_steps=4, guidance=7.5, seed=99)


def _kw(cfg):
    kw = dict(cond=_ids(1, cfg.clip.vocab_size), uncond=_ids(2, cfg.clip.vocab_size))
    if cfg.clip2 is not None:
        kw.update(cond2=_ids(3, cfg.clip2.vocab_size), uncond2=_ids(4, cfg.clip2.vocab_size))
    return kw


def _rank(rank, world, d, port, owners, out):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    from cake_amd.models.sd.config import mini_config
    from cake_amd.sd_engine import NativeSD
    eng = NativeSD(str(d), dtype="f16", autotune=False, rank=rank, world=world,
                   master_addr=f"127.0.0.1:{port}", owners=owners, hop_timeout_s=30.0,
                   connect_timeout_s=60.0)
    info = eng.split_info()
    if rank == 0:
        cfg = mini_config("xl")
        img = eng.generate(**GEN, **_kw(cfg))
        again = eng.generate(**GEN, **_kw(cfg))  # a second generation replays the graphs
        np.savez(out, lat=img.latents, rgb=img.rgb, lat2=again.latents, used=info["ranks_used"],
                 stages=info["stages"])
        eng.close()
    else:
        eng.serve()
        eng.close()


@pytest.fixture(scope="module")
def mini_xl(tmp_path_factory):
    import torch
    from cake_amd.models.sd.config import mini_config
    from cake_amd.models.sd.weights import write_sd_checkpoint
    d = tmp_path_factory.mktemp("sd_mini_split")
    cfg = mini_config("xl")
    write_sd_checkpoint(d, cfg, torch.float16, seed=5, mini=True)
    return cfg, d


@pytest.mark.parametrize("world,owners", [(2, None), (3, None), (2, [0, 0, 0, 0, 1])])
def test_split_unet_matches_single_rank(cuda, mini_xl, tmp_path, world, owners):
    from cake_amd.sd_engine import NativeSD
    cfg, d = mini_xl
    eng = NativeSD(str(d), dtype="f16", autotune=False)
    ref = eng.generate(**GEN, **_kw(cfg))
    eng.close()
    out = tmp_path / "split.npz"
    mp.start_processes(_rank, args=(world, d, _port(), owners, str(out)), nprocs=world,
                       start_method="spawn")
    r = np.load(out)
    assert int(r["used"]) == min(world, int(r["stages"]))
    assert np.array_equal(r["lat"], ref.latents)
    assert np.array_equal(r["rgb"], ref.rgb)
    assert np.array_equal(r["lat2"], ref.latents)
