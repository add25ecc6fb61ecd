"""The simulator's virtual clock (csrc/core/vclock.h, parallel/simclock.py).

With the clock on, counted threads wait in model time: the clock jumps to the
next deadline once every counted thread is blocked, so sleeping an hour of
model time takes no wall time, concurrent sleepers overlap, and a barrier or a
sim session is timed in model seconds."""

import threading
import time

import pytest

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.parallel import simclock


def test_off_is_the_steady_clock():
    assert not _core.vclock_enabled()
    a = _core.vclock_now()
    time.sleep(0.01)
    assert _core.vclock_now() - a >= 0.009


def test_sleepers_overlap_in_model_time_and_cost_no_wall_time():
    with simclock.virtual_clock():
        w0 = time.perf_counter()
        res, span = simclock.run_ranks([lambda: _core.vclock_sleep(3600.0), lambda: _core.vclock_sleep(1800.0),
                                        lambda: (_core.vclock_sleep(600.0), _core.vclock_sleep(600.0))])
        assert span == pytest.approx(3600.0, abs=1e-6)  # concurrent, not 6600 s
        assert time.perf_counter() - w0 < 5.0
    assert not _core.vclock_enabled()


def test_model_time_barrier_releases_together():
    """A VBarrier waits in model time: the rank that sleeps longest decides
    when every rank passes it (a threading.Barrier would hold its waiters
    'busy' and stop the clock)."""
    with simclock.virtual_clock():
        bar = simclock.barrier(3)
        passed = []

        def rank(d):
            _core.vclock_sleep(d)
            bar()
            passed.append(_core.vclock_now())

        _, span = simclock.run_ranks([lambda d=d: rank(d) for d in (1.0, 5.0, 2.0)])
        assert span == pytest.approx(5.0, abs=1e-6)
        assert max(passed) - min(passed) < 1e-9


def test_uncounted_threads_do_not_hold_the_clock():
    """A thread the clock does not count (here: a plain Python thread) never
    stops the clock; counted ones waiting on it would otherwise deadlock."""
    with simclock.virtual_clock():
        stats0 = _core.vclock_stats()
        t = threading.Thread(target=lambda: _core.vclock_sleep(10.0))  # uncounted sleeper
        t.start()
        _, span = simclock.run_ranks([lambda: _core.vclock_sleep(20.0)])
        t.join(5)
        assert not t.is_alive()
        assert span == pytest.approx(20.0, abs=1e-6)
        assert _core.vclock_stats()["advances"] > stats0["advances"]
