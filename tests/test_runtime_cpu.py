"""Native host runtime: wire codec golden bytes, topology semantics, safetensors, split tool."""
import json
import struct
import subprocess

import pytest
import torch

from cake_amd.parallel import proto as P
from cake_amd.parallel.topology import Topology, expand_layer_range
from cake_amd.utils.native import runtime
from cake_amd.utils.safetensors_io import SafeTensors, ShardedCheckpoint, save_file


# ---------------------------------------------------------------- protocol (Appendix A)
def test_hello_frame_golden_bytes():
    assert P.frame({"type": P.HELLO}) == bytes.fromhex("c7f40401" "04000000" "00000000")


def test_batch_golden_bytes_and_roundtrip():
    x = torch.tensor([[1.0, 2.0]], dtype=torch.float32)
    name, shape, buf = P.tensor_payload(x)
    body = P.encode({"type": P.BATCH, "dtype": name, "shape": shape,
                     "batch": [("model.layers.7", 5, 7)]}, buf)
    exp = struct.pack(">I", 3)
    exp += struct.pack(">I", 8) + struct.pack("<2f", 1.0, 2.0)
    exp += struct.pack(">I", 3) + b"f32"
    exp += struct.pack(">I", 2) + struct.pack(">QQ", 1, 2)
    exp += struct.pack(">I", 1) + struct.pack(">I", 14) + b"model.layers.7" + struct.pack(">QQ", 5, 7)
    assert body == exp
    m = P.decode(body)
    assert m["batch"] == [("model.layers.7", 5, 7)] and m["shape"] == [1, 2]
    assert torch.equal(P.tensor_from_payload(m, body), x)


def test_worker_info_and_errors_roundtrip():
    info = {"version": "0.1.0", "dtype": "bf16", "os": "linux", "arch": "x86_64",
            "device": "rocm", "device_idx": 3, "latency": 12}
    m = P.decode(P.encode({"type": P.WORKER_INFO, "info": info}))
    assert m["info"] == info
    m = P.decode(P.encode({"type": P.SINGLE_OP, "layer_name": "unet", "index_pos": 0,
                           "block_idx": 0, "dtype": "u32", "shape": [1, 77]},
                          torch.zeros(77, dtype=torch.int32).numpy().view("uint8")))
    assert m["layer_name"] == "unet" and m["nbytes"] == 308
    assert P.decode(P.encode({"type": P.ERROR, "error": "boom"}))["error"] == "boom"
    assert P.decode(P.encode({"type": P.RESET, "session": 9}))["session"] == 9
    rt = runtime()
    with pytest.raises(Exception):
        rt.decode_header(bytes.fromhex("00000000" "04000000"))  # bad magic
    with pytest.raises(Exception):
        rt.decode_header(struct.pack("<II", rt.PROTO_MAGIC, rt.MESSAGE_MAX_SIZE + 1))
    with pytest.raises(Exception):
        P.decode(b"\x00\x00\x00\x03\x00")  # truncated


# ---------------------------------------------------------------- topology (Appendix C)
def test_range_expansion_rules():
    assert expand_layer_range("model.layers.0-2") == ["model.layers.0", "model.layers.1",
                                                      "model.layers.2"]
    assert expand_layer_range("model.layers.17") == ["model.layers.17"]
    with pytest.raises(Exception):
        expand_layer_range("model.layers.5-5")
    t = Topology.from_text("sd:\n  host: h:1\n  layers:\n    - unet\n    - x.1-3\n",
                           text_model=False)
    assert t["sd"].layers == ["unet", "x.1-3"]  # no expansion for image models


def test_topology_lookup_and_ownership():
    t = Topology.from_text("a:\n  host: 'h:1'\n  layers: ['model.layers.1', 'model.layers.10-11']\n")
    assert t.get_node_for_layer("model.layers.10").name == "a"
    assert t.get_node_for_layer("model.layers.2") is None
    n = t["a"]
    assert n.is_text_model_layer_owner("model.layers.1.mlp.up_proj.weight")
    assert not n.is_text_model_layer_owner("model.layers.12.mlp.up_proj.weight")
    assert Topology.from_text(Topology.from_text(t.to_yaml()).to_yaml()).nodes == t.nodes
    with pytest.raises(Exception):
        Topology.from_text("a:\n  layers: [x]\n")  # host required


# ---------------------------------------------------------------- safetensors + split
def test_safetensors_roundtrip(tmp_path):
    ts = {"a": torch.randn(3, 4), "b": torch.randn(7).to(torch.bfloat16),
          "c": torch.arange(5, dtype=torch.int64), "e": torch.zeros(0)}
    save_file(ts, tmp_path / "m.safetensors", {"format": "pt"})
    f = SafeTensors(tmp_path / "m.safetensors")
    assert sorted(f.keys()) == sorted(ts) and f.metadata() == {"format": "pt"}
    for k, v in ts.items():
        assert torch.equal(f.get(k), v)
    # readable by the reference-compatible python implementation too
    from safetensors.torch import load_file
    other = load_file(str(tmp_path / "m.safetensors"))
    assert all(torch.equal(other[k], v) for k, v in ts.items())
    assert json.loads(runtime().json_roundtrip('{"x":[1,2.5,"\\u00e9"],"y":null}')) == \
        {"x": [1, 2.5, "é"], "y": None}


def test_split_model_tool(tmp_path):
    from cake_amd.build import SPLIT_TOOL
    from cake_amd.utils.synth import tiny_config, write_checkpoint
    src = write_checkpoint(tmp_path / "src", tiny_config(num_hidden_layers=4), torch.float32,
                           shard_bytes=1 << 20)
    topo = tmp_path / "topology.yml"
    topo.write_text("w1:\n  host: '10.0.0.1:10128'\n  layers: ['model.layers.0-1']\n"
                    "w2:\n  host: '10.0.0.2:10128'\n  layers: ['model.layers.3']\n")
    r = subprocess.run([str(SPLIT_TOOL), "--model-path", str(src), "--topology", str(topo),
                        "--output", str(tmp_path / "out")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    full = ShardedCheckpoint(src)
    for w, layers in (("w1", [0, 1]), ("w2", [3])):
        b = tmp_path / "out" / f"{w}-node"
        idx = json.loads((b / "model" / "model.safetensors.index.json").read_text())
        names = sorted(idx["weight_map"])
        expect = sorted(n for n in full.weight_map
                        if any(n.startswith(f"model.layers.{l}.") for l in layers))
        assert names == expect and set(idx["weight_map"].values()) == {"reduced.safetensors"}
        part = ShardedCheckpoint(b / "model")
        for n in names:
            assert torch.equal(part.get(n), full.get(n))
        assert (b / "model" / "config.json").exists()
        t = Topology.from_path(str(b / "topology.yml"))
        assert t.names() == [w]


@pytest.mark.parametrize("entry", [
    {"dtype": "F32", "shape": [2], "data_offsets": [-8, 0]},          # negative begin
    {"dtype": "F32", "shape": [2], "data_offsets": [0, -8]},          # negative end
    {"dtype": "F32", "shape": [-2], "data_offsets": [0, 8]},          # negative dim
    {"dtype": "F32", "shape": [2**62, 8], "data_offsets": [0, 8]},    # numel overflow
    {"dtype": "F32", "shape": [4], "data_offsets": [0, 1 << 40]},     # past the mapping
])
def test_safetensors_rejects_malformed_headers(tmp_path, entry):
    """The native mmap reader validates header integers before forming a view."""
    import struct
    from cake_amd.utils.native import runtime
    hdr = json.dumps({"t": entry}).encode()
    p = tmp_path / "bad.safetensors"
    p.write_bytes(struct.pack("<Q", len(hdr)) + hdr + b"\0" * 16)
    with pytest.raises(Exception):
        runtime().SafeTensorsFile(str(p))
