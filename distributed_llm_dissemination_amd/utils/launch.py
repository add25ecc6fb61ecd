"""Rank -> GPU binding for torchrun launches (one process per GPU).

The normal binding is ``LOCAL_RANK`` (or the config's ``Device``). For
rehearsing multi-rank RCCL schedules on a box with fewer GPUs than ranks,
``DISSEM_SHARED_GPU=1`` binds every rank to device 0 and gives each rank its
own ``NCCL_HOSTID``: RCCL's duplicate-GPU check compares (host hash, bus id),
so distinct host ids make it accept several ranks on one device and route
their traffic over its network transport (sockets on loopback) instead of
xGMI. Functionally identical schedules, chunk matching and CRC verification;
the bandwidth is meaningless and bench output says so.
"""

from __future__ import annotations

import os
import socket
from typing import Dict, Optional

SHARED_ENV = "DISSEM_SHARED_GPU"
# Rehearsal of a multi-node layout on one machine: DISSEM_FAKE_HOSTS=H splits
# the ranks into H "hosts" of world / H consecutive ranks each (host-aware comm
# lanes, hierarchical plans); the transport is still this machine's.
FAKE_HOSTS_ENV = "DISSEM_FAKE_HOSTS"


def shared_gpu() -> bool:
    return os.environ.get(SHARED_ENV, "") == "1"


def rank_device(rank: int, local_rank: int, configured: Optional[int] = None) -> int:
    """Device index for this rank. Must run before the first RCCL call of the process."""
    if shared_gpu():
        os.environ.setdefault("NCCL_HOSTID", f"dissem-shared-gpu-rank{rank}")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        return 0
    return configured if configured is not None else local_rank


def routable_ip() -> str:
    """This machine's address on the interface that reaches MASTER_ADDR (a UDP
    connect sends nothing), else its hostname's address."""
    peer = os.environ.get("MASTER_ADDR", "")
    if peer and peer not in ("127.0.0.1", "localhost"):
        try:
            with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
                s.connect((peer, int(os.environ.get("MASTER_PORT", "29500"))))
                return s.getsockname()[0]
        except OSError:
            pass
    try:
        return socket.gethostbyname(socket.gethostname())
    except OSError:
        return "127.0.0.1"


def gather_hosts(node_id: int) -> Optional[Dict[int, str]]:
    """Multi-node torchrun (process group up): node id -> host name of every
    rank, or None when they all run on this machine. DISSEM_FAKE_HOSTS=H
    pretends the ranks fill H hosts (rehearsal on one machine)."""
    import torch.distributed as dist

    world = dist.get_world_size()
    fake = int(os.environ.get(FAKE_HOSTS_ENV, "0") or 0)
    pairs = [None] * world
    dist.all_gather_object(pairs, (node_id, dist.get_rank(), socket.gethostname()))
    if fake > 1:
        per = max(1, world // fake)
        return {nid: f"host{min(r // per, fake - 1)}" for nid, r, _ in pairs}
    hosts = {nid: h for nid, _, h in pairs}
    return hosts if len(set(hosts.values())) > 1 else None


def listen_addr(multi_host: bool) -> str:
    """Control-plane listen address: loopback on one machine, every interface
    when peers sit on other hosts (advertise it with advertised())."""
    return "0.0.0.0:0" if multi_host and not os.environ.get(FAKE_HOSTS_ENV) else "127.0.0.1:0"


def advertised(addr: str) -> str:
    """The address peers dial for a transport bound to `addr`."""
    host, _, port = addr.rpartition(":")
    return f"{routable_ip()}:{port}" if host in ("0.0.0.0", "") else addr
