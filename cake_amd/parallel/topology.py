"""topology.yml (parsed natively, csrc/runtime/topology.cpp).

Reference: cake-core/src/cake/topology.rs — ``Topology::from_path`` (range
expansion for text models), ``get_node_for_layer`` (exact match),
``Node::is_text_model_layer_owner`` (``"{layer}."`` prefix).
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ..utils.native import runtime


@dataclass
class Node:
    name: str
    host: str
    description: str | None = None
    layers: list[str] = field(default_factory=list)

    def is_text_model_layer_owner(self, full_layer_name: str) -> bool:
        return any(full_layer_name.startswith(f"{p}.") for p in self.layers)


class Topology:
    def __init__(self, nodes: list[Node]):
        self.nodes = nodes
        self._by_name = {n.name: n for n in nodes}

    @classmethod
    def from_text(cls, text: str, text_model: bool = True) -> "Topology":
        return cls([Node(**d) for d in runtime().parse_topology(text, text_model)])

    @classmethod
    def from_path(cls, path: str, text_model: bool = True) -> "Topology":
        return cls([Node(**d) for d in runtime().load_topology(str(path), text_model)])

    @classmethod
    def empty(cls) -> "Topology":
        return cls([])

    def get_node_for_layer(self, layer_name: str) -> Node | None:
        for n in self.nodes:
            if layer_name in n.layers:
                return n
        return None

    def __getitem__(self, name: str) -> Node:
        return self._by_name[name]

    def get(self, name: str) -> Node | None:
        return self._by_name.get(name)

    def __contains__(self, name: str) -> bool:
        return name in self._by_name

    def __len__(self) -> int:
        return len(self.nodes)

    def __iter__(self):
        return iter(self.nodes)

    def names(self) -> list[str]:
        return [n.name for n in self.nodes]

    def to_yaml(self) -> str:
        out = []
        for n in self.nodes:
            out.append(f"{n.name}:\n  host: '{n.host}'\n")
            if n.description is not None:
                out.append(f"  description: '{n.description}'\n")
            out.append("  layers:\n" + "".join(f"  - {l}\n" for l in n.layers))
        return "".join(out)


def expand_layer_range(spec: str) -> list[str]:
    return runtime().expand_layer_range(spec)
