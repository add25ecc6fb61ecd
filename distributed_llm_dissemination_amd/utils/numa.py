"""Host-memory placement next to the GPU (one process per GPU).

On a multi-socket 8-GPU node each GPU's PCIe root port hangs off one socket.
Pinned host layers are the staging source of every host->HBM copy, so a rank
should allocate them on its GPU's NUMA node: otherwise half the ranks' staging
crosses the inter-socket fabric, which all eight ranks then share. The
reference has no equivalent (one process per machine).

``bind_to_gpu(device)`` restricts the calling thread's CPUs to the GPU's node
(threads started later inherit it) and makes that node the preferred one for
its page allocations (set_mempolicy MPOL_PREFERRED), so the pinned pages the
thread faults in land there. Call it before allocating host layers. Anything
that is unknown (no sysfs entry, node -1, a cpuset that excludes the node's
CPUs) leaves the process as it was.
"""

from __future__ import annotations

import ctypes
import os
import platform
from typing import Dict, Optional, Set

_SYS_SET_MEMPOLICY = 238  # x86_64
_MPOL_PREFERRED = 1


def parse_cpulist(text: str) -> Set[int]:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}"""
    out: Set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def pci_bdf(device: int) -> Optional[str]:
    """PCI address 'dddd:bb:dd.0' of a visible GPU (from the torch device properties)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device)
        return f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}.0"
    except Exception:
        return None


def gpu_numa_node(device: int, sysfs: str = "/sys") -> int:
    bdf = pci_bdf(device)
    if bdf is None:
        return -1
    try:
        with open(os.path.join(sysfs, "bus/pci/devices", bdf, "numa_node")) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def node_cpus(node: int, sysfs: str = "/sys") -> Set[int]:
    try:
        with open(os.path.join(sysfs, f"devices/system/node/node{node}/cpulist")) as f:
            return parse_cpulist(f.read())
    except OSError:
        return set()


def _prefer_node(node: int) -> bool:
    if platform.machine() != "x86_64":  # the syscall number below is x86_64's
        return False
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        mask = ctypes.c_ulong(1 << node)
        return libc.syscall(_SYS_SET_MEMPOLICY, _MPOL_PREFERRED, ctypes.byref(mask),
                            ctypes.c_ulong(8 * ctypes.sizeof(mask) + 1)) == 0
    except Exception:
        return False


def bind_to_gpu(device: int) -> Dict[str, int]:
    """Pin this thread's CPUs and page preference to the GPU's NUMA node.

    Returns {"numa_node", "cpus", "mempolicy"} describing what was applied
    ({} when nothing was); DISSEM_NUMA_BIND=0 turns it off, DISSEM_NUMA_NODE=k
    binds to node k instead (A/B runs: a deliberately remote node)."""
    if os.environ.get("DISSEM_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return {}
    forced = os.environ.get("DISSEM_NUMA_NODE", "")
    node = int(forced) if forced else gpu_numa_node(device)
    if node < 0 or node >= 64:
        return {}
    cpus = node_cpus(node) & os.sched_getaffinity(0)
    if not cpus:
        return {}
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        return {}
    return {"numa_node": node, "cpus": len(cpus), "mempolicy": int(_prefer_node(node))}
