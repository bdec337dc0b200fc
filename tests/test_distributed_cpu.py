"""Master/worker over the framed TCP transport on localhost (CPU, f32).

Equivalence invariant: any topology reproduces the all-local greedy token stream,
also across consecutive requests (worker KV reset — SURVEY Appendix E Q7)."""
import pytest
import torch

from cake_amd.cli import build_parser
from cake_amd.context import Context
from cake_amd.models.chat import Message
from cake_amd.models.llama3.generator import LLamaGenerator
from cake_amd.parallel import proto as P
from cake_amd.parallel.client import Client, RemoteError
from cake_amd.parallel.worker import Worker
from cake_amd.utils.synth import tiny_config, write_checkpoint


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = tmp_path_factory.mktemp("tiny4")
    write_checkpoint(d, tiny_config(num_hidden_layers=4), torch.float32, shard_bytes=1 << 20)
    return d


def _ctx(ckpt, topo_path, *extra):
    args = build_parser().parse_args(["--model", str(ckpt), "--topology", str(topo_path), "--cpu",
                                      "--temperature", "0", *extra])
    return Context.from_args(args)


def _start_worker(ckpt, tmp_path, name, layers):
    topo = tmp_path / f"{name}.yml"
    topo.write_text(f"{name}:\n  host: '127.0.0.1:0'\n  layers:\n" +
                    "".join(f"    - {l}\n" for l in layers))
    w = Worker(_ctx(ckpt, topo, "--mode", "worker", "--name", name, "--address", "127.0.0.1:0"))
    w.serve_in_thread()
    return w


def _generate(ctx, prompts, n=12):
    gen = LLamaGenerator.load(ctx)
    outs = []
    for p in prompts:
        gen.reset()
        gen.add_message(Message.system("sys"))
        gen.add_message(Message.user(p))
        toks = gen.stream(n, lambda t: None, stop_at_eos=False)
        outs.append([t.id for t in toks])
    return outs


def test_topology_equivalence_and_reset(ckpt, tmp_path):
    empty = tmp_path / "empty.yml"
    empty.write_text("{}\n")
    prompts = ["The sky is blue because", "Tell me a story about a very long road"]
    local = _generate(_ctx(ckpt, empty), prompts)
    w1 = _start_worker(ckpt, tmp_path, "w1", ["model.layers.1-2"])
    w2 = _start_worker(ckpt, tmp_path, "w2", ["model.layers.3"])
    try:
        topo = tmp_path / "topology.yml"
        topo.write_text(f"w1:\n  host: '127.0.0.1:{w1.port}'\n  layers:\n    - 'model.layers.1-2'\n"
                        f"w2:\n  host: '127.0.0.1:{w2.port}'\n  description: 'tail'\n"
                        f"  layers: [model.layers.3]\n")
        ctx = _ctx(ckpt, topo)
        gen = LLamaGenerator.load(ctx)
        runs = [(r.ident, r.layers) for r in gen.model.runs]
        assert runs == [("local", [0]), (f"127.0.0.1:{w1.port}", [1, 2]),
                        (f"127.0.0.1:{w2.port}", [3])]
        dist = _generate(ctx, prompts)
        assert dist == local
    finally:
        w1.stop()
        w2.stop()


def test_worker_errors_and_ping(ckpt, tmp_path):
    w = _start_worker(ckpt, tmp_path, "w", ["model.layers.0"])
    try:
        c = Client("cpu", f"127.0.0.1:{w.port}", "model.layers.0")
        assert c.info["device"] == "cpu" and c.info["version"] == P.PROTO_VERSION
        c.ping()
        x = torch.randn(1, 3, 256)
        y = c.forward_batch(x, [("model.layers.0", 0, 0)])
        assert y.shape == x.shape and not torch.equal(x, y)
        with pytest.raises(RemoteError):
            c.forward_batch(x, [("model.layers.3", 0, 3)])  # not served here
        c.reset()
        y2 = c.forward_mut(x, 0, 0)
        assert torch.allclose(y, y2)
        c.close()
    finally:
        w.stop()


def test_unknown_worker_name_serves_first_node(ckpt, tmp_path):
    topo = tmp_path / "t.yml"
    topo.write_text("a:\n  host: '127.0.0.1:0'\n  layers: [model.layers.0]\n"
                    "b:\n  host: '127.0.0.1:0'\n  layers: [model.layers.1]\n")
    w = Worker(_ctx(ckpt, topo, "--mode", "worker", "--name", "nope", "--address", "127.0.0.1:0"))
    try:
        assert w.node.name == "a" and w.stack.layer_ids == [0]
    finally:
        w.stop()


def test_fault_injection_and_native_stats(ckpt, tmp_path, monkeypatch):
    monkeypatch.setenv("CAKE_FAULT_INJECT", "drop_after=2")
    w = _start_worker(ckpt, tmp_path, "wf", ["model.layers.0"])
    try:
        c = Client("cpu", f"127.0.0.1:{w.port}", "model.layers.0")
        x = torch.randn(1, 1, 256)
        c.forward_mut(x, 0, 0)
        c.forward_mut(x, 1, 0)           # 2nd op: the worker then drops the connection
        with pytest.raises(Exception):
            c.forward_mut(x, 2, 0)
        st = w.stats()
        assert st["ops"] == 2 and st["connections"] == 1 and st["bytes_in"] > 0
    finally:
        w.stop()


def test_loopback_transport_matches_local(ckpt, tmp_path):
    """--transport loopback: every topology node served in-process over the wire protocol
    reproduces the all-local greedy stream."""
    from cake_amd.parallel.loopback import start_loopback_workers, stop_loopback_workers
    local = _generate(_ctx(ckpt, tmp_path / "none.yml"), ["hello"], n=8)
    topo = tmp_path / "loop.yml"
    topo.write_text("a:\n  host: 'unused:1'\n  layers:\n    - model.layers.0-1\n"
                    "b:\n  host: 'unused:2'\n  layers:\n    - model.layers.3\n")
    ctx = _ctx(ckpt, topo, "--transport", "loopback")
    workers = start_loopback_workers(ctx)
    try:
        assert all(n.host.startswith("127.0.0.1:") for n in ctx.topology.nodes)
        assert _generate(ctx, ["hello"], n=8) == local
        assert sum(w.stats()["ops"] for w in workers) > 0
    finally:
        stop_loopback_workers(workers)
