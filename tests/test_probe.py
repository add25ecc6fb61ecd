"""Untimed pre-flight link probe (Runtime.probe_links -> PlannedEngine.probe),
on the simulated fabric: every directed pair on its own lane at once, then
each pair alone; a lane whose partner never posts is named, not waited on."""

import itertools
import threading

import pytest

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.models.catalog import make_workload
from distributed_llm_dissemination_amd.parallel.runtime import Runtime

MiB = 1 << 20
_keys = itertools.count()


def _cluster(n, timing=None):
    key = f"probe{next(_keys)}"
    cfg = make_workload(n, n, MiB, tier="host", seeding="random", chunk_bytes=MiB)
    bar = threading.Barrier(n)
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key,
                   barrier=bar.wait) for i in range(n)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    if timing is not None:
        _core.sim_set_timing(key, timing)
    return rts


def _all(rts, fn):
    out = [None] * len(rts)
    err = [None] * len(rts)

    def go(i):
        try:
            out[i] = fn(rts[i])
        except Exception as e:  # noqa: BLE001
            err[i] = e

    ths = [threading.Thread(target=go, args=(i,)) for i in range(len(rts))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    return out, err


@pytest.mark.parametrize("n", [2, 4, 8])
def test_probe_measures_every_directed_link(n):
    t = _core.SimTiming()
    t.link_bps = 2.5e8  # slow enough that the modelled time dominates host copy overheads under load
    t.link = {(0, 1): 6.25e7}  # one slow directed link
    rts = _cluster(n, t)
    try:
        out, err = _all(rts, lambda r: r.probe_links(4 * MiB, timeout_s=20))
        assert err == [None] * n, err
        for r, o in enumerate(out):
            peers = {p for p in range(n) if p != r}
            assert set(o["concurrent"]) == peers and set(o["solo"]) == peers
        slow = out[0]["solo"][1]
        fast = [out[a]["solo"][b] for a in range(n) for b in range(n) if a != b and (a, b) != (0, 1)]
        fast.sort()
        assert slow < 0.5 * fast[len(fast) // 2], (slow, fast)  # a quarter-rate link, against the median
        # the probe leaves the engine ready for sessions
        res, err = _all(rts, lambda r: (r.prepare(1), r.execute(30))[1])
        assert all(x.ok for x in res), [x.error for x in res]
    finally:
        for r in rts:
            r.close()


def test_probe_names_a_stalled_lane():
    """Rank 1 never posts its side: rank 0's lanes to and from it stall and the
    probe raises after its timeout, naming them (bench.py then fails the
    attempt and its supervisor starts the fallback)."""
    t = _core.SimTiming()
    t.wait_s = 1.0  # the fabric gives up on the never-matched sends after 1 s (default 30), so close() returns
    rts = _cluster(2, t)
    try:
        rts[0]._barrier = lambda: None
        with pytest.raises(RuntimeError, match=r"stalled after 0 s on node 0: lane \d+ \(send to node 1\)"):
            rts[0].probe_links(MiB, timeout_s=0.5, solo=False)
    finally:
        rts[1].close()
        rts[0].close()
