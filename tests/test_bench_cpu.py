"""bench.py contract on CPU: self-launched N>1 ranks (no torchrun), fail-fast on a dead rank.

The driver runs ``bench.py --gpus N`` (torchrun or bare); without WORLD_SIZE in the
environment bench.py spawns the ranks itself.  --cpu runs the reference math with gloo
so the launch / aggregation / equivalence plumbing is covered without a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--cpu", "--model", "tiny", "--steps", "5", "--warmup", "2", "--prompt-len", "9",
        "--max-seq", "64"]


def _run(extra, env=None, timeout=240):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, "bench.py", *ARGS, *extra], cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout, env=e)


def _json(r):
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-2000:]
    return json.loads(lines[0])


def test_self_launch_matches_single(tmp_path):
    r1 = _run(["--dump-tokens", str(tmp_path / "a.json")])
    assert r1.returncode == 0, r1.stderr[-2000:]
    r2 = _run(["--gpus", "3", "--parallel", "pp", "--dump-tokens", str(tmp_path / "b.json")])
    assert r2.returncode == 0, r2.stderr[-2000:]
    j = _json(r2)
    assert j["n_gpus"] == 3 and j["steps"] == 5 and j["warmup"] == 2 and j["value"] > 0
    assert j["config"]["global_batch"] == 1 and j["scaling"] == "strong"
    assert j["hops_per_token"] == 3 and j["hop_us"] > 0
    a = json.loads((tmp_path / "a.json").read_text())
    b = json.loads((tmp_path / "b.json").read_text())
    assert a[0] == b[0]          # layer sharding does not change the token stream


def test_self_launch_fails_fast_when_a_rank_dies():
    r = _run(["--gpus", "3", "--parallel", "pp"], env={"CAKE_BENCH_FAIL_RANK": "2"}, timeout=120)
    assert r.returncode != 0
    assert "stopping the others" in r.stderr


def test_default_multi_rank_headline_is_layer_sharding():
    """N > 1 without --parallel: the reference's layer sharding is the headline."""
    r = _run(["--gpus", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json(r)
    assert j["n_gpus"] == 2 and j["config"]["parallelism"].startswith("pp2")
    assert j["parallel"] == "pp" and j["hops_per_token"] == 2


def test_self_launch_tensor_parallel(tmp_path):
    """--parallel tp: tensor-parallel ranks; same stream at TP 1 and TP 2 is covered
    by tests/test_tp_cpu.py (here: the launch / JSON contract)."""
    r = _run(["--gpus", "2", "--parallel", "tp", "--model", "tiny-kv2",
              "--dump-tokens", str(tmp_path / "t.json")])
    assert r.returncode == 0, r.stderr[-2000:]
    j = _json(r)
    assert j["n_gpus"] == 2 and j["config"]["parallelism"].startswith("tp2")
    assert j["allreduces_per_token"] == 2 * 2 + 1 and j["value"] > 0
    toks = json.loads((tmp_path / "t.json").read_text())[0]
    assert len(toks) == 9 + 1 + 2 + 5   # prompt + first token + warmup + timed steps


def test_eight_ranks_full_extras_tiny():
    """The full default N>1 bench path at N = 8 on the tiny presets (--tiny-extras):
    headline pp, tp (skipped: 8 does not divide tiny-kv2's KV heads), pp_streams,
    the 70B pp / tp sub-records and the split-UNet SD sub-record — the code the
    driver's 8-GPU run executes, end to end on gloo."""
    import time
    t0 = time.time()
    r = _run(["--gpus", "8", "--tiny-extras", "--sd-steps", "2"], timeout=600)
    wall = time.time() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json(r)
    assert j["n_gpus"] == 8 and j["config"]["parallelism"].startswith("pp8")
    assert "skipped" in j["tp"]
    assert j["pp_streams"]["tokens_per_sec"] > 0
    assert j["llama3_70b"]["pp"]["tokens_per_sec"] > 0
    assert "tokens_per_sec" in j["llama3_70b"]["tp"] or "skipped" in j["llama3_70b"]["tp"]
    sd = j["sd"]["sdxl_tiny_split"]
    n_stages = sum(len(v) for v in sd["stages"].values())   # tiny SDXL: 5 block groups
    assert sd["ranks_used"] == min(8, n_stages) and sd["seconds_per_step"] > 0, sd
    assert sd["hops_per_step"] == sd["ranks_used"] and len(sd["compute_s_per_rank"]) == 8
    assert wall < 600
    print(f"8-rank tiny full bench wall {wall:.1f}s")


def test_split_sd_matches_single_rank():
    """The split-UNet steps give the same latents as the whole UNet on one rank (CPU f32,
    gloo, one OpenMP thread per rank): the packed hops carry the feature map and the
    skip stack exactly."""
    env = {"OMP_NUM_THREADS": "1"}
    r1 = _run(["--tiny-extras", "--sd-steps", "2"], env={**env, "WORLD_SIZE": "1", "RANK": "0",
                                                           "MASTER_PORT": "29731"}, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r3 = _run(["--gpus", "3", "--tiny-extras", "--sd-steps", "2"], env=env, timeout=400)
    assert r3.returncode == 0, r3.stderr[-3000:]
    a = _json(r1)["sd"]["sdxl_tiny_split"]
    b = _json(r3)["sd"]["sdxl_tiny_split"]
    assert a["ranks_used"] == 1 and b["ranks_used"] == 3
    assert a["latent_checksum"] == b["latent_checksum"] and a["latent_abs"] == b["latent_abs"]
