"""Stable Diffusion over the device transport on the GPU (ranks share cuda:0; gloo for
the process group, CAKE_DIST_BACKEND=gloo).  (a) an SDXL-shaped tiny UNet split by block
group over two worker ranks gives the single-rank image (per-step path on both sides);
(b) a UNet whole on one worker runs the fused graph-replayed denoising loop there and
gives the single-rank (fused) image."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, cwd, extra_env):
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0",
               CAKE_DIST_BACKEND="gloo", CAKE_SERVE_IDLE_TIMEOUT="120", **extra_env)
    env.pop("WORLD_SIZE", None)
    try:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=150, env=env, cwd=cwd)
    except subprocess.TimeoutExpired as e:  # name the stuck rank's last words
        err = e.stderr.decode(errors="replace") if isinstance(e.stderr, bytes) else e.stderr
        pytest.fail(f"timed out: {' '.join(cmd[-6:])}\n{(err or '')[-3000:]}")


@pytest.mark.timeout(400)
@pytest.mark.parametrize("version,topo,n,fused", [
    ("xl", "w1:\n  host: 'r1'\n  layers: ['unet.down']\n"
           "w2:\n  host: 'r2'\n  layers: ['unet.mid', 'unet.up', 'vae']\n", 3, "0"),
    ("v1-5", "w1:\n  host: 'r1'\n  layers: ['unet', 'clip']\n", 2, "1"),
])
def test_sd_rccl_gpu_matches_local(cuda, tmp_path, version, topo, n, fused):
    from cake_amd.models.sd.config import tiny_config
    from cake_amd.models.sd.weights import write_sd_checkpoint
    d = tmp_path / "sd"
    write_sd_checkpoint(d, tiny_config(version), torch.float16, tiny=True)
    (tmp_path / "empty.yml").write_text("{}\n")
    (tmp_path / "t.yml").write_text(topo)
    common = ["--model", str(d), "--model-type", "image-model", "--sd-version", version,
              "--sd-image-prompt", "a rusty robot", "--sd-n-steps", "4", "--sd-seed", "5",
              "--sd-guidance-scale", "7.5"]
    env = {"CAKE_SD_FUSED_STEP": fused, "CAKE_CONV_AUTOTUNE": "0"}
    (tmp_path / "local").mkdir()
    (tmp_path / "dist").mkdir()
    r = _run([sys.executable, "-m", "cake_amd.cli", "--topology", str(tmp_path / "empty.yml"),
              *common], tmp_path / "local", env)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
              f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
              "-m", "cake_amd.cli", "--transport", "rccl", "--topology", str(tmp_path / "t.yml"),
              *common], tmp_path / "dist", env)
    first_tb = r.stderr.find("Traceback")
    assert r.returncode == 0, r.stderr[max(0, first_tb):][:4000] + "\n...\n" + r.stderr[-1500:]
    # the two runs are separate processes: MIOpen's algorithm choice for the tiny model's
    # 32-channel convolutions may differ between them, so pixels agree to rounding, not
    # bit for bit (a misrouted hop or skip tensor changes the image wholesale)
    import numpy as np
    from PIL import Image
    a = np.asarray(Image.open(tmp_path / "local" / "images" / "image_0_0.png"), dtype=np.int16)
    b = np.asarray(Image.open(tmp_path / "dist" / "images" / "image_0_0.png"), dtype=np.int16)
    assert a.shape == b.shape
    d = np.abs(a - b)
    assert d.mean() < 1.0 and (d > 8).mean() < 0.005, (d.mean(), d.max(), (d > 8).mean())
