"""Elastic recovery of the planned (RCCL) data plane, on the simulated fabric.

A rank dies in the middle of a session (fault injection: it stops posting after
a few P2P groups and its control endpoint disappears). The survivors' groups
with it stall; they report the peers (Suspect), the leader's liveness probe
finds the dead rank, every survivor shrinks the communicator around it
(the RCCL path is ncclCommShrink with NCCL_SHRINK_ABORT) and the leader
re-plans what was not acked from live holders. The session completes for the
survivors, byte-exact; the dead rank's own assignment is dropped and counted.
The reference has no failure handling at all.
"""

import itertools
import threading

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.models.catalog import make_workload
from distributed_llm_dissemination_amd.parallel.runtime import Runtime, layer_seed

MiB = 1 << 20
_keys = itertools.count()


def _holders(cfg, layer):
    return {nd.id for nd in cfg.nodes for per in nd.initial_layers.values() if layer in per}


def _cluster(cfg, dead_rank, die_after, mode=1, **policy):
    key = f"recov{next(_keys)}"
    n = len(cfg.nodes)
    rts = []
    for i in range(n):
        opts = {"suspect_s": 0.5}
        if i == dead_rank:
            opts["inject_die_after_groups"] = die_after
        rts.append(Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key,
                           engine_opts=opts))
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for r in rts:
            r.prepare(mode, **policy)
        res = [None] * n

        def go(i):
            res[i] = rts[i].execute(6 if i == dead_rank else 60)

        ths = [threading.Thread(target=go, args=(i,)) for i in range(n)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        sizes = cfg.layer_sizes()
        for i, r in enumerate(rts):
            if i == dead_rank:
                continue
            assert res[i].ok, (i, res[i].error)
            for l in cfg.assignment.get(i, []):
                if _holders(cfg, l) == {dead_rank}:
                    continue  # lost with its only holder
                assert r.layer_bytes(l) == _core.fill_random_host(sizes[l], layer_seed(0, l)), (i, l)
        return res, rts
    finally:
        for r in rts:
            r.close()


def test_rank_death_mid_session_shrinks_and_completes():
    cfg = make_workload(4, 8, 4 * MiB, tier="host", seeding="uniform", copies=2, seed=1, chunk_bytes=MiB)
    res, _ = _cluster(cfg, dead_rank=3, die_after=2)
    leader = res[0]
    assert leader.recoveries == 1
    assert leader.dropped == len(cfg.assignment[3])  # the dead rank's own layers
    shrinks = [r.engine_stats.get("shrinks", 0) for r in res[:3]]
    assert shrinks == [1, 1, 1]
    assert not res[3].ok


def test_rank_death_mode2_pull_schedule():
    cfg = make_workload(4, 8, 3 * MiB, tier="host", seeding="uniform", copies=2, seed=2, chunk_bytes=MiB)
    res, _ = _cluster(cfg, dead_rank=2, die_after=3, mode=2, pull_window=3)
    assert res[0].recoveries == 1


def test_layer_without_live_holder_is_dropped():
    # copies=1: the dead rank's seeded layers have no other holder; the survivors
    # still finish everything else and the lost pairs are counted.
    cfg = make_workload(3, 6, 2 * MiB, tier="host", seeding="uniform", copies=1, seed=4, chunk_bytes=MiB)
    lost = [l for l in range(6) if _holders(cfg, l) == {2}]
    assert lost
    res, _ = _cluster(cfg, dead_rank=2, die_after=1)
    assert res[0].recoveries == 1
    # the dead rank's own assignment + every survivor's copy of a lost layer
    assert res[0].dropped == len(cfg.assignment[2]) + 2 * len(lost)


def test_false_alarm_does_not_shrink():
    """A tiny suspect timeout makes ordinary groups look stalled: ranks report
    suspects, the leader's probe finds every peer alive, nothing is shrunk and
    the session completes normally."""
    key = f"recov{next(_keys)}"
    cfg = make_workload(3, 6, 4 * MiB, tier="host", seeding="random", chunk_bytes=MiB)
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key,
                   engine_opts={"suspect_s": 1e-4}) for i in range(3)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for r in rts:
            r.prepare(1)
        res = [None] * 3
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(30))) for i in range(3)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert all(x.ok for x in res), [x.error for x in res]
        assert res[0].recoveries == 0 and res[0].dropped == 0
        assert all(x.engine_stats["shrinks"] == 0 for x in res)
    finally:
        for r in rts:
            r.close()


def test_rank_death_eight_ranks_mode3_flow():
    # mode 3 stripes layers over several senders in byte ranges; after the
    # shrink the leader re-plans the unacked layers whole from live holders.
    cfg = make_workload(8, 16, 4 * MiB, tier="host", seeding="uniform", copies=3, seed=3, chunk_bytes=MiB)
    res, _ = _cluster(cfg, dead_rank=5, die_after=2, mode=3)
    assert res[0].recoveries == 1
    assert res[0].dropped == len(cfg.assignment[5])


def test_rank_death_on_two_hosts_hierarchical():
    """2 hosts x 4 GPUs (host-aware lanes, hierarchical mode 1 with imports and
    xGMI relays): a rank of the second host dies mid-session. The survivors
    drop to per-distance lanes over the shrunk communicator and the leader's
    re-plan still imports once per host - every survivor ends byte-exact."""
    cfg = make_workload(8, 16, 4 * MiB, tier="host", seeding="uniform", copies=2, seed=5, chunk_bytes=MiB)
    for nd in cfg.nodes:
        nd.host = f"h{nd.id // 4}"
    res, _ = _cluster(cfg, dead_rank=6, die_after=2, owner_policy="links")
    assert res[0].recoveries == 1
    assert res[0].dropped == len(cfg.assignment[6])
