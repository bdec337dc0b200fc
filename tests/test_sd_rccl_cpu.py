"""Stable Diffusion over the device transport (parallel/sd_rccl.py) on the CPU: torchrun
ranks with gloo.  The images equal the single-process generation when (a) the UNet is
split by block group over two worker ranks and the VAE sits on a third, (b) the UNet
is whole on one worker and CLIP on another."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from cake_amd.models.sd.config import tiny_config
from cake_amd.models.sd.weights import write_sd_checkpoint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, cwd):
    # torchrun gives each rank one OpenMP thread: the single-process reference must use
    # the same count, or CPU matmul reduction order differs (bits, not transport)
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=cwd)


@pytest.mark.parametrize("version,topo,n", [
    ("xl", "w1:\n  host: 'r1'\n  layers: ['unet.down']\n"
           "w2:\n  host: 'r2'\n  layers: ['unet.mid', 'unet.up']\n"
           "w3:\n  host: 'r3'\n  layers: ['vae']\n", 4),
    ("v1-5", "w1:\n  host: 'r1'\n  layers: ['unet']\n"
             "w2:\n  host: 'r2'\n  layers: ['clip', 'unet.up.2']\n", 3),
])
def test_sd_rccl_matches_local(tmp_path, version, topo, n):
    d = tmp_path / "sd"
    write_sd_checkpoint(d, tiny_config(version), torch.float32, tiny=True)
    (tmp_path / "empty.yml").write_text("{}\n")
    (tmp_path / "t.yml").write_text(topo)
    common = ["--model", str(d), "--cpu", "--model-type", "image-model", "--sd-version", version,
              "--sd-image-prompt", "a rusty robot", "--sd-n-steps", "3", "--sd-seed", "5",
              "--sd-guidance-scale", "7.5"]
    (tmp_path / "local").mkdir()
    (tmp_path / "dist").mkdir()
    r = _run([sys.executable, "-m", "cake_amd.cli", "--topology", str(tmp_path / "empty.yml"),
              *common], tmp_path / "local")
    assert r.returncode == 0, r.stderr[-3000:]
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
              f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
              "-m", "cake_amd.cli", "--transport", "rccl", "--topology", str(tmp_path / "t.yml"),
              *common], tmp_path / "dist")
    assert r.returncode == 0, r.stderr[-4000:]
    a = (tmp_path / "local" / "images" / "image_0_0.png").read_bytes()
    b = (tmp_path / "dist" / "images" / "image_0_0.png").read_bytes()
    assert a == b
