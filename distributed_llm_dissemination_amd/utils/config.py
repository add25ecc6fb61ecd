"""Topology config: the reference's JSON schema, parsed strictly.

Reference: cmd/config.go:14-62 (schema + ReadJson), readme.md:16-63 (older flat
schema). Both forms are accepted:

* nested (current code): ``"InitialLayers": {"<SourceType>": {"<LayerID>": {"LayerSize": n}}}``
* flat (README):          ``"InitialLayers": {"<LayerID>": {}}`` with the top-level ``LayerSize``

Go's encoding/json matches keys case-insensitively ("Id" == "ID"); so do we.
Unlike the reference (quirk Q15), malformed files raise instead of yielding an
empty config.

Extensions (all optional): per node ``"Device"`` (GPU ordinal) and ``"Host"``
(the machine the node's GPU sits in: GPUs of one host share its xGMI mesh,
hosts are joined by the network; default: one host), top-level ``"Links"``
(``{"<src>": {"<dst>": bytes_per_s}}`` directed link bandwidths for the
topology-aware planners) and ``"ChunkBytes"``.
"""

from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

# SourceType (distributor/node.go:192-198) + the HBM extension.
SOURCE_CLIENT, SOURCE_DISK, SOURCE_MEM, SOURCE_DEVICE = 0, 1, 2, 3
CLIENT_ID = (1 << 64) - 1  # distributor/client.go:10


class ConfigError(ValueError):
    pass


def _get(obj: Dict[str, Any], key: str, default: Any = None) -> Any:
    if key in obj:
        return obj[key]
    low = key.lower()
    for k, v in obj.items():
        if k.lower() == low:
            return v
    return default


def _int(v: Any, what: str) -> int:
    if isinstance(v, bool) or not isinstance(v, (int, float, str)):
        raise ConfigError(f"{what}: expected an integer, got {v!r}")
    try:
        return int(v)
    except ValueError as e:
        raise ConfigError(f"{what}: expected an integer, got {v!r}") from e


@dataclass
class NodeConf:
    id: int
    addr: str = ""
    network_bw: int = 0
    is_leader: bool = False
    sources: Dict[int, int] = field(default_factory=dict)  # source type -> rate (B/s)
    initial_layers: Dict[int, Dict[int, int]] = field(default_factory=dict)  # source -> layer -> size
    device: Optional[int] = None
    host: Optional[str] = None

    def layer_ids(self) -> List[int]:
        return sorted({l for per in self.initial_layers.values() for l in per})


@dataclass
class ClientConf:
    id: int  # the node this client serves
    addr: str = ""
    layers: Dict[int, int] = field(default_factory=dict)  # layer -> rate (B/s)


@dataclass
class Config:
    nodes: List[NodeConf]
    clients: List[ClientConf] = field(default_factory=list)
    assignment: Dict[int, List[int]] = field(default_factory=dict)
    layer_size: int = 0
    links: Dict[int, Dict[int, int]] = field(default_factory=dict)
    chunk_bytes: Optional[int] = None

    # cmd/config.go:64-92
    def leader(self) -> NodeConf:
        for n in self.nodes:
            if n.is_leader:
                return n
        raise ConfigError("no leader found")

    def node(self, node_id: int) -> NodeConf:
        for n in self.nodes:
            if n.id == node_id:
                return n
        raise ConfigError(f"node {node_id} not found in config")

    def client(self, node_id: int) -> Optional[ClientConf]:
        for c in self.clients:
            if c.id == node_id:
                return c
        return None

    def network_bw(self) -> Dict[int, int]:
        return {n.id: n.network_bw for n in self.nodes}

    def hosts(self) -> Dict[int, int]:
        """node id -> host group (0, 1, ... in order of first appearance); every
        node on host 0 when no node names its Host."""
        groups: Dict[str, int] = {}
        return {n.id: groups.setdefault(n.host or "", len(groups)) for n in self.nodes}

    def registry(self) -> Dict[int, str]:
        return {n.id: n.addr for n in self.nodes}

    def layer_sizes(self) -> Dict[int, int]:
        sizes: Dict[int, int] = {}
        for n in self.nodes:
            for per in n.initial_layers.values():
                for l, s in per.items():
                    sizes[l] = max(sizes.get(l, 0), s)
        for c in self.clients:
            for l in c.layers:
                sizes.setdefault(l, self.layer_size)
        for layers in self.assignment.values():
            for l in layers:
                sizes.setdefault(l, self.layer_size)
        return sizes

    def to_json(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {
            "Nodes": [
                {
                    "Id": n.id,
                    "Addr": n.addr,
                    "NetworkBW": n.network_bw,
                    "IsLeader": n.is_leader,
                    "Sources": {str(k): v for k, v in n.sources.items()},
                    "InitialLayers": {
                        str(st): {str(l): {"LayerSize": s} for l, s in per.items()}
                        for st, per in n.initial_layers.items()
                    },
                    **({"Device": n.device} if n.device is not None else {}),
                    **({"Host": n.host} if n.host is not None else {}),
                }
                for n in self.nodes
            ],
            "Assignment": {str(k): {str(l): {} for l in v} for k, v in self.assignment.items()},
            "LayerSize": self.layer_size,
        }
        if self.clients:
            out["Clients"] = [
                {"ID": c.id, "Addr": c.addr, "Layers": {str(l): r for l, r in c.layers.items()}}
                for c in self.clients
            ]
        if self.links:
            out["Links"] = {str(s): {str(d): bw for d, bw in v.items()} for s, v in self.links.items()}
        if self.chunk_bytes:
            out["ChunkBytes"] = self.chunk_bytes
        return out


def _is_nested(initial: Dict[str, Any]) -> bool:
    # Nested when some value is an object whose values are themselves objects.
    for v in initial.values():
        if isinstance(v, dict) and any(isinstance(x, dict) for x in v.values()):
            return True
    return False


def parse_config(raw: Dict[str, Any]) -> Config:
    if not isinstance(raw, dict):
        raise ConfigError("config must be a JSON object")
    layer_size = _int(_get(raw, "LayerSize", 0) or 0, "LayerSize")
    nodes_raw = _get(raw, "Nodes")
    if not isinstance(nodes_raw, list) or not nodes_raw:
        raise ConfigError("config has no Nodes")
    # Schema form is decided per file: nested if any node uses the nested form, or
    # if there is no top-level LayerSize (the flat form sizes layers by it).
    nested_file = any(
        isinstance(nr, dict) and isinstance(_get(nr, "InitialLayers"), dict) and _is_nested(_get(nr, "InitialLayers"))
        for nr in nodes_raw
    ) or not layer_size
    nodes: List[NodeConf] = []
    for i, nr in enumerate(nodes_raw):
        if not isinstance(nr, dict):
            raise ConfigError(f"Nodes[{i}] is not an object")
        nid = _int(_get(nr, "ID", _get(nr, "Id")), f"Nodes[{i}].ID")
        sources = {
            _int(k, "Sources key"): _int(v, "Sources value") for k, v in (_get(nr, "Sources", {}) or {}).items()
        }
        init_raw = _get(nr, "InitialLayers", {}) or {}
        if not isinstance(init_raw, dict):
            raise ConfigError(f"Nodes[{i}].InitialLayers must be an object")
        initial: Dict[int, Dict[int, int]] = {}
        if nested_file:
            for st, per in init_raw.items():
                layers: Dict[int, int] = {}
                for lid, lconf in (per or {}).items():
                    size = _int(_get(lconf or {}, "LayerSize", layer_size) or 0, "LayerSize")
                    layers[_int(lid, "LayerID")] = max(size, 0)  # negative sizes clamp to 0 (config.go:99-102)
                initial[_int(st, "SourceType")] = layers
        else:
            # README flat form: layer ids, sized by the global LayerSize, held in memory.
            flat = {_int(lid, "LayerID"): max(layer_size, 0) for lid in init_raw}
            if flat:
                initial[SOURCE_MEM] = flat
        dev = _get(nr, "Device")
        host = _get(nr, "Host")
        nodes.append(
            NodeConf(
                id=nid,
                addr=str(_get(nr, "Addr", "") or ""),
                network_bw=_int(_get(nr, "NetworkBW", 0) or 0, "NetworkBW"),
                is_leader=bool(_get(nr, "IsLeader", False)),
                sources=sources,
                initial_layers=initial,
                device=None if dev is None else _int(dev, "Device"),
                host=None if host is None else str(host),
            )
        )
    ids = [n.id for n in nodes]
    if len(set(ids)) != len(ids):
        raise ConfigError(f"duplicate node ids: {ids}")
    clients = []
    for i, cr in enumerate(_get(raw, "Clients", []) or []):
        clients.append(
            ClientConf(
                id=_int(_get(cr, "ID", _get(cr, "Id")), f"Clients[{i}].ID"),
                addr=str(_get(cr, "Addr", "") or ""),
                layers={_int(k, "layer"): _int(v, "rate") for k, v in (_get(cr, "Layers", {}) or {}).items()},
            )
        )
    assignment: Dict[int, List[int]] = {}
    for k, v in (_get(raw, "Assignment", {}) or {}).items():
        if isinstance(v, dict):
            layers = [_int(l, "Assignment layer") for l in v]
        elif isinstance(v, list):
            layers = [_int(l, "Assignment layer") for l in v]
        else:
            raise ConfigError(f"Assignment[{k}] must be an object or list")
        assignment[_int(k, "Assignment node")] = sorted(layers)
    links = {
        _int(s, "Links src"): {_int(d, "Links dst"): _int(bw, "Links bw") for d, bw in per.items()}
        for s, per in (_get(raw, "Links", {}) or {}).items()
    }
    cb = _get(raw, "ChunkBytes")
    cfg = Config(nodes=nodes, clients=clients, assignment=assignment, layer_size=layer_size, links=links,
                 chunk_bytes=None if cb is None else _int(cb, "ChunkBytes"))
    cfg.leader()  # must exist
    for nid in assignment:
        cfg.node(nid)
    return cfg


def load_config(path: str) -> Config:
    with open(path, "r", encoding="utf-8") as f:
        try:
            raw = json.load(f)
        except json.JSONDecodeError as e:
            raise ConfigError(f"failed to load json file: {path}: {e}") from e
    return parse_config(raw)


def example_config(n: int = 4, layer_size: int = 1 << 20) -> Config:
    """What the reference's disabled PrintJsonExample meant to print (cmd/config.go:200-249)."""
    nodes = [NodeConf(id=i, addr=f":{8080 + i}", is_leader=(i == 0)) for i in range(n)]
    nodes[0].initial_layers = {SOURCE_MEM: {1: layer_size, 3: layer_size}}
    if n > 1:
        nodes[1].initial_layers = {SOURCE_MEM: {1: layer_size}}
    if n > 3:
        nodes[3].initial_layers = {SOURCE_MEM: {3: layer_size}}
    assignment = {1: [1], 2: [1, 3], 3: [3]} if n > 3 else {i: [1] for i in range(1, n)}
    return Config(nodes=nodes, assignment=assignment, layer_size=layer_size)
