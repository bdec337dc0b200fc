"""Split-UNet steps on device hops (parallel/sd_split.py _DeviceChannels over
parallel/hop.py BulkInbox / BulkPeer, csrc/kernels/hop.hip bulk kernels).

Ranks share cuda:0 (RCCL refuses duplicate GPUs: gloo carries the first, eager step's
packed messages and the setup; every later step is one hipGraph replay per rank whose
hops are IPC peer stores + flags).  The latents equal the whole UNet on one rank, the
routed packed path (CAKE_SD_SPLIT_DEVICE=0) agrees too, and a receive with no sender
times out into the error word instead of hanging."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _split(n: int, extra_env=None) -> dict:
    args = ["bench.py", "--model", "tiny", "--steps", "3", "--warmup", "2", "--prompt-len", "9",
            "--max-seq", "128", "--tiny-extras", "--extras", "sd", "--sd-steps", "3"]
    # fixed convolution plans: the autotuner may pick a different (differently rounded)
    # variant per process, which would make bitwise equality across runs luck
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CAKE_HOP_TIMEOUT="30",
               CAKE_CONV_AUTOTUNE="0", **(extra_env or {}))
    if n > 1:
        args += ["--gpus", str(n), "--dist-backend", "gloo", "--launch-timeout", "200"]
        env.pop("WORLD_SIZE", None)
    else:
        env.update(WORLD_SIZE="1", RANK="0", MASTER_PORT="29761")
    r = subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True,
                       timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)["sd"]["sdxl_tiny_split"]


def test_split_unet_device_hops_match_single_rank(cuda):
    one = _split(1)
    assert one["ranks_used"] == 1
    packed = _split(3, {"CAKE_SD_SPLIT_DEVICE": "0"})
    assert "packed buffer per hop" in packed["transport"]
    assert packed["latent_checksum"] == one["latent_checksum"], (packed, one)
    three = _split(3)
    assert three["ranks_used"] == 3 and three["transport"].startswith("device bulk hops"), three
    assert three["latent_checksum"] == one["latent_checksum"], (three, one)
    assert three["latent_abs"] == one["latent_abs"]
    assert three["hop_bytes"] and all(v > 0 for v in three["hop_bytes"].values())
    # skips routed straight to their consumer: some channel skips the next rank
    assert any(int(k.split("->")[1]) - int(k.split("->")[0]) > 1
               for k in three["channels"]), three["channels"]


def test_bulk_receive_times_out_into_error_word(cuda):
    from cake_amd.parallel.hop import BulkInbox
    box = BulkInbox(4096, "cuda:0")
    dst = torch.empty(4096, dtype=torch.uint8, device="cuda:0")
    box.recv(dst, timeout_s=0.2)
    torch.cuda.synchronize()
    assert box.error()
    assert int(box.seq.item()) == 1  # the receive still advanced: later ones fail fast
    box.close()
