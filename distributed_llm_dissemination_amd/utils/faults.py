"""Fault-injection specs (the reference has no fault handling).

``--inject`` takes one or more comma-free specs::

    drop-chunk=P         every received chunk is damaged with probability P
                         behind its P2P group (planned engines); the CRC check
                         catches it, the receiver NACKs, the leader re-sends
    kill-rank=R@T        node R exits abruptly T seconds after it starts
                         sending layer bytes (host engines: the leader's job deadline
                         re-dispatches its jobs; planned engines: the survivors'
                         group watchdog reports it, the leader probes and the
                         survivors abort and re-form the communicators without it,
                         then the leader re-plans - elastic recovery)
    slow-link=S:D:RATE   sender S paces layer bytes to D at RATE B/s (host
                         engine: per-connection token bucket; planned engines:
                         the issue thread's per-link bucket; K/M/G suffixes are
                         powers of 1000)
    fail-attempt=R@K     bench.py supervised runs (N > 1): rank R's worker fails
                         right after its process group forms in attempt K, so
                         the supervisors stop every worker and start the next,
                         fallback attempt (utils/supervise.py)

Several specs may be given (``--inject drop-chunk=0.01 --inject kill-rank=3@2``).
"""

from __future__ import annotations

import os
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

_SUFFIX = {"": 1, "K": 10**3, "M": 10**6, "G": 10**9}


def parse_rate(s: str) -> int:
    s = s.strip().upper().replace("/S", "").rstrip("B")
    unit = s[-1] if s and s[-1] in _SUFFIX else ""
    num = s[: len(s) - len(unit)] if unit else s
    return int(float(num) * _SUFFIX[unit])


@dataclass
class FaultPlan:
    drop_chunk: float = 0.0
    kill: Dict[int, float] = field(default_factory=dict)  # node id -> seconds after session start
    slow_links: Dict[Tuple[int, int], int] = field(default_factory=dict)  # (src, dst) -> B/s
    fail_attempts: Dict[int, List[int]] = field(default_factory=dict)  # rank -> supervised attempts it fails

    def link_rates_from(self, node_id: int) -> Dict[int, int]:
        return {d: r for (s, d), r in self.slow_links.items() if s == node_id}


def parse_inject(specs: Optional[List[str]]) -> FaultPlan:
    plan = FaultPlan()
    for spec in specs or []:
        if "=" not in spec:
            raise ValueError(f"bad --inject spec {spec!r} (want kind=value)")
        kind, val = spec.split("=", 1)
        kind = kind.strip().lower()
        if kind == "drop-chunk":
            p = float(val)
            if not 0.0 <= p <= 1.0:
                raise ValueError("drop-chunk probability must be in [0, 1]")
            plan.drop_chunk = p
        elif kind == "kill-rank":
            if "@" not in val:
                raise ValueError("kill-rank wants R@T (node id @ seconds)")
            r, t = val.split("@", 1)
            plan.kill[int(r)] = float(t)
        elif kind == "slow-link":
            parts = val.split(":")
            if len(parts) != 3:
                raise ValueError("slow-link wants S:D:RATE")
            plan.slow_links[(int(parts[0]), int(parts[1]))] = parse_rate(parts[2])
        elif kind == "fail-attempt":
            if "@" not in val:
                raise ValueError("fail-attempt wants R@K (rank @ attempt index)")
            r, k = val.split("@", 1)
            plan.fail_attempts.setdefault(int(r), []).append(int(k))
        else:
            raise ValueError(f"unknown --inject kind {kind!r}")
    return plan


def arm_kill(plan: FaultPlan, node_id: int, started: Optional[Callable[[], bool]] = None) -> Optional[threading.Thread]:
    """Start the kill timer for this node if the plan names it (call at session start).

    With `started`, the T seconds count from the moment it first returns True
    (e.g. the node has begun sending layer bytes) rather than from the call, so
    the fault lands mid-transfer however long the other processes take to start.
    """
    if node_id not in plan.kill:
        return None
    delay = plan.kill[node_id]

    def die() -> None:
        if started is not None:
            while not started():
                time.sleep(0.005)
        time.sleep(delay)
        print(f'{{"level":"warn","node":{node_id},"message":"fault injection: kill-rank fired"}}',
              file=sys.stderr, flush=True)
        os._exit(86)  # abrupt: no goodbye to peers, sockets reset

    t = threading.Thread(target=die, daemon=True)
    t.start()
    return t
