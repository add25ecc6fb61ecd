"""Model-time harness for in-process simulations (csrc/core/vclock.h).

With the virtual clock on, the simulated fabric, the engines' queues and polls,
the token buckets and the node's event loop wait in model time: the clock
jumps to the next deadline as soon as every thread it counts is blocked, so a
session's length is its modeled makespan - identical run to run and on an idle
or a loaded host - and nothing sleeps on the wall clock.

The Python threads that run a session's ranks must be counted too (a rank's
thread between its announce and its wait is work the clock must not skip
past): ``run_ranks`` reserves them before they start and each adopts its
reservation. Threads the clock does not count must not block on something a
counted thread waits for - use ``barrier(n)`` rather than threading.Barrier.
"""

from __future__ import annotations

import contextlib
import threading
from typing import Callable, List, Sequence, Tuple

from .. import _core


@contextlib.contextmanager
def virtual_clock():
    """Run the block in model time (nested uses share the outer one)."""
    if _core.vclock_enabled():
        yield
        return
    _core.vclock_enable(True)
    try:
        yield
    finally:
        _core.vclock_enable(False)


def now() -> float:
    """Model time in seconds (the steady clock when the virtual clock is off)."""
    return _core.vclock_now()


def barrier(n: int) -> Callable[[], None]:
    """A barrier for n rank threads that waits in model time."""
    return _core.VBarrier(n).wait


def run_ranks(fns: Sequence[Callable[[], object]], wall_timeout_s: float = 900.0) -> Tuple[List[object], float]:
    """Run every fn in its own thread, all counted by the clock; returns their
    results and the span from the start to the last one's return (seconds of
    model time with the virtual clock on, else wall time). Raises the first
    exception a fn raised."""
    n = len(fns)
    res: List[object] = [None] * n
    errs: List[BaseException] = []
    ends = [0.0] * n
    counted = _core.vclock_enabled()
    if counted:
        _core.vclock_reserve(n)  # the clock cannot move until every thread has started
    t0 = _core.vclock_now()

    def go(i):
        if counted:
            _core.vclock_adopt()
        try:
            res[i] = fns[i]()
        except BaseException as e:  # noqa: BLE001 - re-raised by the caller
            errs.append(e)
        finally:
            ends[i] = _core.vclock_now()  # before release: idle timers may move the clock after it
            if counted:
                _core.vclock_release()

    ths = [threading.Thread(target=go, args=(i,), daemon=True) for i in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(wall_timeout_s)
        if t.is_alive():
            raise RuntimeError(f"simulated ranks still running after {wall_timeout_s:.0f} s of wall time "
                               f"(clock: {_core.vclock_describe() if counted else 'off'})")
    if errs:
        raise errs[0]
    return res, max(ends) - t0 if n else 0.0
