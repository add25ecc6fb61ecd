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
from typing import Optional

SHARED_ENV = "DISSEM_SHARED_GPU"


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
