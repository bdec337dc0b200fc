"""Which image topologies the native engine's split UNet serves (parallel/sd_rccl.py
native_split_owners): UNet stages only, in contiguous runs over ranks 0, 1, 2, ... in stage
order; a text encoder or the VAE on a worker rank, another order, or nothing placed keeps
the Python transport."""
from cake_amd.models.sd.config import get_config
from cake_amd.parallel.sd_rccl import native_split_owners
from cake_amd.parallel.topology import Topology

XL = get_config("xl")  # 3 down blocks: down.0-2, mid, up.0-2


def _topo(text):
    return Topology.from_text(text, text_model=False)


def test_up_path_on_rank_one():
    t = _topo("w1:\n  host: 'a:1'\n  layers: ['unet.up']\n")
    assert native_split_owners(t, XL, 2) == [0, 0, 0, 0, 1, 1, 1]


def test_three_runs():
    t = _topo("w1:\n  host: 'a:1'\n  layers: ['unet.mid', 'unet.up.0']\n"
              "w2:\n  host: 'b:1'\n  layers: ['unet.up.1', 'unet.up.2']\n")
    assert native_split_owners(t, XL, 3) == [0, 0, 0, 1, 1, 2, 2]


def test_python_transport_cases():
    # the VAE on a worker, stages out of order, nothing placed
    assert native_split_owners(_topo("w1:\n  host: 'a:1'\n  layers: ['vae', 'unet.up']\n"),
                               XL, 2) is None
    assert native_split_owners(_topo("w1:\n  host: 'a:1'\n  layers: ['unet.down.0']\n"),
                               XL, 2) is None
    assert native_split_owners(_topo("w1:\n  host: 'a:1'\n  layers: ['unet.up.2']\n"
                                     "w2:\n  host: 'b:1'\n  layers: ['unet.up.1']\n"),
                               XL, 3) is None
    assert native_split_owners(Topology.empty(), XL, 2) is None
