"""Workload catalog: layer-shard shapes of real models and synthetic topologies.

The reference's only experiment is ``conf/config.json`` (8 nodes, 8 layers of
10.93 GB, all assigned to node 7). BASELINE.json names the MI355X targets:
80 x 1 GiB (Llama-3-70B-sized shards) and 126 x 3 GiB (Llama-3.1-405B-sized),
delivered to 1/2/4/8 ranks of one node. ``make_workload`` turns such a shape
plus a seeding policy into a reference-schema Config.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from ..utils.config import SOURCE_DEVICE, SOURCE_DISK, SOURCE_MEM, Config, NodeConf

GiB = 1 << 30
MiB = 1 << 20


@dataclass(frozen=True)
class ModelShards:
    name: str
    layers: int
    layer_bytes: int
    note: str = ""


CATALOG: Dict[str, ModelShards] = {
    "llama3-70b": ModelShards("llama3-70b", 80, 1 * GiB, "80 decoder layers; BASELINE configs #2-#4"),
    "llama3.1-405b": ModelShards("llama3.1-405b", 126, 3 * GiB, "126 decoder layers; BASELINE config #5 (fp8 wire)"),
    "reference-ec2": ModelShards("reference-ec2", 8, 10_930_691_768, "reference conf/config.json"),
    "tiny": ModelShards("tiny", 4, 1 * MiB, "BASELINE config #1 (CPU loopback)"),
}

TIER_SOURCE = {"host": SOURCE_MEM, "mem": SOURCE_MEM, "disk": SOURCE_DISK, "device": SOURCE_DEVICE, "hbm": SOURCE_DEVICE}


def seed_owners(layers: int, ranks: int, copies: int = 1, seed: int = 0, balanced: bool = True) -> Dict[int, List[int]]:
    """Random InitialLayers seeding: layer -> the ranks holding it.

    ``balanced`` shuffles the layers and deals them round-robin, so every rank
    holds layers*copies/ranks of them (random *which*, equal *how many*);
    otherwise each layer picks its holders uniformly at random.
    """
    rng = np.random.default_rng(seed)
    copies = max(1, min(copies, ranks))
    owners: Dict[int, List[int]] = {}
    if balanced:
        perm = rng.permutation(layers)
        for pos, layer in enumerate(perm):
            base = pos % ranks
            owners[int(layer)] = sorted({(base + k * max(1, ranks // copies)) % ranks for k in range(copies)})
    else:
        for layer in range(layers):
            owners[layer] = sorted(int(x) for x in rng.choice(ranks, size=copies, replace=False))
    return owners


def make_workload(
    ranks: int,
    layers: int,
    layer_bytes: int,
    *,
    seeding: str = "random",
    tier: str = "host",
    copies: int = 1,
    seed: int = 0,
    assignment: str = "replicate",
    network_bw: int = 0,
    tier_rate: int = 0,
    base_port: int = 0,
    chunk_bytes: Optional[int] = None,
) -> Config:
    """Build a reference-schema Config.

    seeding:    "random" (balanced random, BASELINE #3), "leader" (all layers on rank 0,
                BASELINE #2), "uniform" (unbalanced random)
    tier:       where seeded copies live: host (pinned RAM), disk (NVMe files), device (HBM)
    assignment: "replicate" (every rank needs every layer) or "pipeline" (rank r needs
                the r-th contiguous block of layers, a PP stage layout)
    """
    st = TIER_SOURCE[tier]
    if seeding == "leader":
        owners = {l: [0] for l in range(layers)}
    else:
        owners = seed_owners(layers, ranks, copies, seed, balanced=(seeding == "random"))
    nodes = []
    for r in range(ranks):
        held = {l: layer_bytes for l, os_ in owners.items() if r in os_}
        nodes.append(
            NodeConf(
                id=r,
                addr=f"127.0.0.1:{base_port + r}" if base_port else "",
                network_bw=network_bw,
                is_leader=(r == 0),
                sources={st: tier_rate},
                initial_layers={st: held} if held else {},
            )
        )
    if assignment == "replicate":
        assign = {r: list(range(layers)) for r in range(ranks)}
    elif assignment == "pipeline":
        assign = {}
        for r in range(ranks):
            lo, hi = r * layers // ranks, (r + 1) * layers // ranks
            assign[r] = list(range(lo, hi))
    else:
        raise ValueError(f"unknown assignment {assignment}")
    return Config(nodes=nodes, assignment=assign, layer_size=layer_bytes, chunk_bytes=chunk_bytes)


def delivered_bytes(cfg: Config) -> int:
    """Bytes that must land in target memory: every assigned (node, layer) not seeded on device."""
    sizes = cfg.layer_sizes()
    total = 0
    for nid, layers in cfg.assignment.items():
        node = cfg.node(nid)
        on_dev = set(node.initial_layers.get(SOURCE_DEVICE, {}))
        total += sum(sizes[l] for l in layers if l not in on_dev)
    return total
