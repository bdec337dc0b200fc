"""The native multi-rank bench falls back to the torch.distributed transport when the native
group cannot start (its start-up IPC self-test failed, or any rank's start threw): every
rank agrees, runs the Python engine over gloo / RCCL, and the record names the transport
("engine": "python", "hop"/"allreduce": "dist") and the native error.

CPU plumbing: gloo, world 2, the native engine replaced by one that raises the engine's
self-test error (the GPU form of the same test forces the real self-test to fail with
CAKE_IPC_SELFTEST_FAIL=1: tests/test_engine_gpu.py)."""
import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, mode, model, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "OMP_NUM_THREADS": "1"})
    sys.path.insert(0, ROOT)
    import bench
    import cake_amd.engine as E
    from cake_amd.parallel.native_bench import measure_native_multi
    from cake_amd.parallel.pipeline_bench import DistEnv

    class Refused:
        def __init__(self, *a, **k):
            raise RuntimeError("pipeline IPC self-test failed: rank 1: forced (test)")

    E.NativeLlama = Refused
    a = bench._args(["--cpu", "--model", model, "--steps", "3", "--warmup", "1",
                     "--prompt-len", "9", "--max-seq", "64", "--gpus", str(world),
                     "--parallel", mode])
    env = DistEnv(a)
    import torch.distributed as dist
    try:
        r = measure_native_multi(a, env, model, 3, 1, mode)
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump(r, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,model", [("pp", "tiny"), ("tp", "tiny-kv2")])
def test_native_group_falls_back_to_dist(tmp_path, mode, model):
    out = tmp_path / "r.json"
    mp.start_processes(_rank, args=(2, _port(), mode, model, str(out)), nprocs=2,
                       start_method="spawn")
    r = json.loads(out.read_text())
    assert r["engine"] == "python" and r["tokens_per_sec"] > 0
    assert "self-test failed" in r["native_fallback"]
    if mode == "pp":
        assert r["hop"] == "dist"
    else:
        assert r["allreduce"] == "dist"
