"""`--transport rccl` master/worker roles (torchrun, one rank per device; gloo on CPU here):
the CLI generation through the rank pipeline equals the all-local generation."""
import os
import subprocess
import sys

import torch

from cake_amd.utils.synth import tiny_config, write_checkpoint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, **kw):
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, **kw)


def test_rccl_roles_match_local(tmp_path):
    d = tmp_path / "m"
    write_checkpoint(d, tiny_config(num_hidden_layers=4), torch.float32)
    (tmp_path / "empty.yml").write_text("{}\n")
    topo = tmp_path / "t.yml"
    topo.write_text("w1:\n  host: 'rank1'\n  layers: ['model.layers.1-2']\n"
                    "w2:\n  host: 'rank2'\n  layers: ['model.layers.3']\n")
    common = ["--model", str(d), "--cpu", "-n", "10", "--temperature", "0", "--prompt", "hi there"]
    local = _run([sys.executable, "-m", "cake_amd.cli", "--topology", str(tmp_path / "empty.yml"),
                  *common])
    assert local.returncode == 0, local.stderr[-2000:]
    dist = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
                 "--master-addr=127.0.0.1", "--master-port=29571", "-m", "cake_amd.cli",
                 "--transport", "rccl", "--topology", str(topo), "--metrics",
                 str(tmp_path / "m.jsonl"), *common])
    assert dist.returncode == 0, dist.stderr[-3000:]
    text = local.stdout.strip()
    assert text and text in dist.stdout
    # metrics sink: hop latency, hops per token and every rank's entry
    import json
    rec = json.loads((tmp_path / "m.jsonl").read_text().splitlines()[-1])
    assert rec["kind"] == "text" and rec["generated"] == 10
    assert rec["hop_us"] is not None and rec["hop_us"] > 0
    assert rec["hops_per_token"] == 3
    assert [r["rank"] for r in rec["rank_hbm"]] == [0, 1, 2]
    assert [r["layers"] for r in rec["rank_hbm"]] == [1, 2, 1]


def test_rccl_tensor_parallel_roles_match_local(tmp_path):
    """--transport rccl --parallel tp: 2 ranks, each 1/2 of every layer (real checkpoint
    slices), rank 0 the master; the CLI text equals the all-local generation."""
    d = tmp_path / "m"
    write_checkpoint(d, tiny_config(num_hidden_layers=3, num_key_value_heads=2), torch.float32)
    (tmp_path / "empty.yml").write_text("{}\n")
    common = ["--model", str(d), "--cpu", "-n", "10", "--temperature", "0", "--prompt", "hi there",
              "--topology", str(tmp_path / "empty.yml")]
    local = _run([sys.executable, "-m", "cake_amd.cli", *common])
    assert local.returncode == 0, local.stderr[-2000:]
    tp = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", "--master-port=29573", "-m", "cake_amd.cli",
               "--transport", "rccl", "--parallel", "tp", *common])
    assert tp.returncode == 0, tp.stderr[-3000:]
    text = local.stdout.strip()
    assert text and text in tp.stdout
