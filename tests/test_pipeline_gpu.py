"""Multi-process pipeline on ONE GPU (host-staged gloo hops; RCCL refuses duplicate GPUs).

Runs bench.py under torchrun with 2 and 3 ranks sharing cuda:0 and checks that the
generated token ids equal the single-rank run (equivalence invariant)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, n, streams, name):
    out = tmp_path / f"{name}.json"
    args = ["bench.py", "--model", "tiny", "--steps", "12", "--warmup", "3", "--prompt-len", "9",
            "--max-seq", "256", "--dump-tokens", str(out)]
    if n == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={29600 + n}",
               ] + args + ["--gpus", str(n), "--dist-backend", "gloo", "--streams", str(streams)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line), json.loads(out.read_text())


def test_pipeline_multirank_matches_single(cuda, tmp_path):
    _, single = _bench(tmp_path, 1, 1, "single")
    m2, pp2 = _bench(tmp_path, 2, 1, "pp2")
    assert pp2[0] == single[0]
    assert m2["n_gpus"] == 2 and m2["value"] > 0
    m3, pp3 = _bench(tmp_path, 3, 2, "pp3")
    assert pp3[0] == single[0]          # stream 0 uses the same prompt as the single run
    assert len(pp3) == 2 and len(pp3[1]) == len(pp3[0])
