"""Schedules under the simulated fabric's timing and RCCL models (CPU).

SimTiming gives the sim fabric per-link bandwidth, per-rank staging (PCIe)
bandwidth and, optionally, RCCL's round-by-round P2P execution. These tests
check what the byte-exact tests in test_planned_sim.py cannot: that lanes keep
irregular groups safe under RCCL's round model, that token-bucket pacing holds
configured rates (reference writeWithLimit, transport.go:407-424; mode-3
size/T rates, node.go:1281; tier LimitRate on self loads, node.go:1615-1624),
and what the headline schedule's T(N) is predicted to be.
"""

import itertools
import os
import sys
import threading
import time

import pytest

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.models.catalog import make_workload
from distributed_llm_dissemination_amd.parallel.runtime import Runtime

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import predict_scaling  # noqa: E402

MiB = 1 << 20
_keys = itertools.count()


@pytest.fixture(scope="module", autouse=True)
def _warm_simulator():
    """The first 8-rank session of a process runs ~1.5x slower (thread and
    allocator warm-up); the timing comparisons below must not depend on order."""
    predict_scaling.predict(8, layers=16, scale=1024, steps=1, slowdown=4)


def run_timed(cfg, mode, timing=None, lanes=0, chunk=MiB, verify=True, **policy):
    key = f"tsim{os.getpid()}_{next(_keys)}"
    if timing is not None:
        _core.sim_set_timing(key, timing)
    n = len(cfg.nodes)
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=chunk, sim_key=key, verify=verify,
                   engine_opts={"lanes": lanes}) for i in range(n)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for r in rts:
            r.prepare(mode, **policy)
        res = [None] * n

        def go(i):
            res[i] = rts[i].execute(60)

        ths = [threading.Thread(target=go, args=(i,)) for i in range(n)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        assert all(x.ok for x in res), [x.error for x in res]
        return dt, res
    finally:
        for r in rts:
            r.close()


def test_lanes_keep_irregular_groups_safe_under_rccl_rounds():
    """Mode 2 at 8 ranks dispatches jobs as acks return, so ranks form
    different groups. Under RCCL's round model (a group's ops run one ring
    distance at a time) a multi-distance group can wait on itself across ranks
    - the 8-rank hang first seen on the GPU box with one lane. With world-1
    lanes every group holds one distance and the session completes."""
    cfg = make_workload(8, 16, 4 * MiB, tier="host", seeding="random", chunk_bytes=MiB)
    t = _core.SimTiming()
    t.p2p_rounds = True
    for _ in range(2):
        _, res = run_timed(cfg, 2, t, lanes=0, pull_window=2)
        assert res[0].engine_stats["verify_failures"] == 0


def test_tier_rate_paces_staging():
    """A host tier with a LimitRate (config Sources) is staged no faster than
    that rate: 8 MiB at 40 MB/s takes ~0.18 s instead of ~0 (the bucket's
    burst of one chunk goes at once, like x/time/rate's initial burst)."""
    rate = 40_000_000
    cfg = make_workload(1, 4, 2 * MiB, tier="host", tier_rate=rate, chunk_bytes=MiB)
    dt, res = run_timed(cfg, 1)
    want = 7 * MiB / rate
    assert want * 0.9 <= dt <= want * 1.5 + 0.1, (dt, want)
    assert res[0].engine_stats["paced"] > 0


def test_mode3_jobs_finish_at_the_planned_T():
    """Mode 3 paces every job at size/T (node.go:1281): with the leader's 50 MB/s
    NetworkBW as the binding cut, the transfers end together close to T."""
    cfg = make_workload(4, 4, 2 * MiB, tier="host", seeding="leader", network_bw=50_000_000, chunk_bytes=MiB // 4)
    dt, res = run_timed(cfg, 3, chunk=MiB // 4)
    T = res[0].flow_T
    assert T == pytest.approx(3 * 4 * 2 * MiB / 50e6, rel=0.02)
    assert abs(dt - T) <= 0.1 * T + 0.05, (dt, T)
    assert res[0].engine_stats["paced"] > 0


def test_mode3_hbm_ingress_budget_binds_the_plan():
    """The mode-3 graph's per-GPU HBM ingress cap (prepare(hbm_gbps=...),
    SURVEY C13'): with every dest's ingress at 20 MB/s and no other limit,
    T is the busiest dest's bytes / 20 MB/s, and the paced jobs finish there."""
    cfg = make_workload(3, 3, 2 * MiB, tier="host", seeding="leader", chunk_bytes=MiB // 4)
    dt, res = run_timed(cfg, 3, chunk=MiB // 4, hbm_gbps=0.02)
    T = res[0].flow_T
    assert T == pytest.approx(3 * 2 * MiB / 20e6, rel=0.02)
    assert abs(dt - T) <= 0.15 * T + 0.05, (dt, T)


def test_predicted_scaling_follows_the_link_bound():
    """The headline schedule on the timing model (scripts/predict_scaling.py)
    at 1/1024 size: T(N) stays within 35 % of the closed form
    85.9 GB / (N * min(PCIe, link)) - the schedule keeps every GPU's PCIe
    copy and its N-1 links busy together (sim thread overhead included)."""
    for n in (1, 2, 4):
        r = predict_scaling.predict(n, scale=1024, link_gbps=50.0, pcie_gbps=57.5, steps=1, slowdown=4)
        bound = 85.899e9 / n / (min(57.5, 50.0 if n > 1 else 1e9) * 1e9)
        assert r["ms_per_step"] / 1e3 <= bound * 1.35, (n, r, bound)
        assert r["ms_per_step"] / 1e3 >= bound * 0.95, (n, r, bound)


def test_slow_link_costs_at_most_a_seventh_with_the_link_aware_plan():
    """One directed link at half speed (8 ranks, headline mode 1, 1/1024 size,
    timing slowed 16x so thread overhead stays out). Lanes are per directed link, so the slow link holds back
    only its own transfers; the leader's link-aware plan (owner policy
    "links" with the config's Links) then moves chunk slices of the layers it
    carries onto relays - ranks that receive the same layer directly - until
    the slowest link no longer sets the pace: <= 1/7 extra time, where a plan
    that ignores the link takes ~2x."""
    kw = dict(layers=32, scale=1024, link_gbps=50.0, pcie_gbps=57.5, mode=1, steps=2, slowdown=16,
              policy={"owner_policy": "links"})
    base = predict_scaling.predict(8, **kw)["ms_per_step"]
    slow = predict_scaling.predict(8, slow_link=((0, 1), 0.5), adapt_links=False, **kw)["ms_per_step"]
    planned = predict_scaling.predict(8, slow_link=((0, 1), 0.5), plan_links=True, adapt_links=False, **kw)["ms_per_step"]
    assert slow > 1.5 * base, (base, slow)
    assert planned <= base * (1 + 1 / 7), (base, planned, slow)


def test_client_stream_cut_through_to_peers():
    """C17 pipe at chunk grain on the GPU data plane: node 1's external client
    streams layer 9 at 20 MB/s; nodes 0 and 2 need it from node 1 over 20 MB/s
    links. Node 1 stages and forwards each chunk as soon as it has landed in
    host memory (transport.go:144-196 tees the TCP stream the same way), so the
    session ends ~one stream time after the start - not stream + forward."""
    from distributed_llm_dissemination_amd.parallel.runtime import layer_seed
    from distributed_llm_dissemination_amd.utils.config import ClientConf

    size, rate = 8 * MiB, 20_000_000
    cfg = make_workload(3, 1, size, tier="host", seeding="leader", chunk_bytes=MiB)
    cfg.clients.append(ClientConf(id=1, addr="", layers={9: rate}))
    cfg.assignment = {r: [9] for r in range(3)}
    key = f"tsim{os.getpid()}_{next(_keys)}"
    t = _core.SimTiming()
    t.link_bps = rate
    _core.sim_set_timing(key, t)
    data = _core.fill_random_host(size, layer_seed(0, 9))
    ct = _core.tcp_transport("127.0.0.1:0", {}, True)
    client = _core.ClientNode(1, ct, {9: _core.LayerSrc.inmem(data, rate)})
    client.start()
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key) for i in range(3)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for i, r in enumerate(rts):
        r.transport.set_registry({**reg, _core.CLIENT_ID: ct.address()} if i == 1 else reg)
    ct.set_registry({1: reg[1]})
    try:
        for r in rts:
            r.prepare(1)
        res = [None] * 3
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(30))) for i in range(3)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        assert all(x.ok for x in res), [x.error for x in res]
        for r in rts:
            assert r.layer_bytes(9) == data
        stream = (size - 256 * 1024) / rate  # the client's token bucket starts with a 256 KiB burst
        assert dt < stream + 0.5 * size / rate, (dt, stream)  # store-and-forward would need stream + size/rate
    finally:
        for r in rts:
            r.close()
        client.stop()
        ct.close()


def test_closed_loop_routes_around_an_unconfigured_slow_link():
    """Closed-loop link rates (Runtime.link_report): one directed link runs at
    half speed and NOTHING in the config or the plan says so. The first session
    pays for it (~2x: the slow link holds back its share); every rank folds its
    per-link busy throughput into an EWMA and announces it, so the leader's
    second plan relays around the slow link: <= 1/7 extra time (reference
    analog: node.go:774-793 times jobs, :1044-1053 steers by those times)."""
    kw = dict(layers=32, scale=1024, link_gbps=50.0, pcie_gbps=57.5, mode=1, slowdown=16,
              policy={"owner_policy": "links"})
    base = predict_scaling.predict(8, steps=2, **kw)["ms_per_step"]
    r = predict_scaling.predict(8, slow_link=((0, 1), 0.5), steps=3, **kw)
    first, *later = r["times_ms"]
    assert first > 1.5 * base, (base, r)
    # both later sessions plan on the measured rates; the better one (thread
    # scheduling of the 8 simulated ranks adds a few % of noise) is within 1/7
    assert min(later) <= base * (1 + 1 / 7), (base, r)
    plan = r["plan_link_GBps_last"]
    assert plan["0->1"] < 0.7 * plan["1->0"], plan  # the leader planned on the measured slow link


def test_closed_loop_replans_mode3_on_faster_links():
    """Mode 3 plans T - and paces every job at size/T (node.go:1281) - from its
    link rates. The plan starts from a constant 40 GB/s while the fabric
    delivers 56 (1.4x): session 1 is paced to the pessimistic T. The measured
    rates feed session 2's plan, whose T is lower, and the paced jobs finish
    within 10 % of it."""
    r = predict_scaling.predict(4, layers=16, scale=1024, link_gbps=56.0, plan_link_gbps=40.0, pcie_gbps=200.0,
                                mode=3, steps=3, slowdown=4, plan_links=True)
    T1, T2, T3 = r["flow_T_ms"]
    t1, t2, t3 = r["times_ms"]
    assert T2 < 0.85 * T1 and T3 < 0.85 * T1, r
    # sessions 2 and 3 both plan on measured rates; the better one (the
    # simulator's thread scheduling adds a few % of noise) ends within 10 % of its T
    t, T = min((t2, T2), (t3, T3))
    assert abs(t - T) <= 0.10 * T, r
    assert t < t1, r


def test_node_shared_disk_budget_paces_every_rank(tmp_path):
    """One NVMe per node (config #4 at N > 1): the ranks' disk readers draw from
    one node-wide budget (engine/node_pacer.h, shared memory): 4 ranks loading
    8 x 1 MiB at a 20 MB/s node rate take ~0.42 s in total, not 1/4 of it."""
    cfg = make_workload(4, 8, MiB, tier="disk", seeding="random", chunk_bytes=MiB // 4)
    key = f"disk{os.getpid()}_{next(_keys)}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB // 4, sim_key=key,
                   storage_path=str(tmp_path), node_disk_gbps=0.02, node_key=key) for i in range(4)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for r in rts:
            r.prepare(1)
        res = [None] * 4
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(60))) for i in range(4)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        assert all(x.ok for x in res), [x.error for x in res]
        want = 8 * MiB / 20e6
        assert want * 0.85 <= dt <= want * 1.5 + 0.2, (dt, want)
        assert sum(x.engine_stats["disk_wait_ms"] for x in res) > 0
    finally:
        for r in rts:
            r.close()


def test_predicted_disk_tier_is_bound_by_the_node_nvme():
    """predict_scaling --tier disk: at N = 4 the headline workload from NVMe is
    bound by the node's single device (80 GiB / 13.3 GB/s = 6.46 s), not by
    N x per-GPU staging."""
    r = predict_scaling.predict(4, scale=4096, steps=1, slowdown=4, tier="disk", layers=16)
    bound = 16 * (1 << 30) / 13.3e9
    assert bound * 0.9 <= r["ms_per_step"] / 1e3 <= bound * 1.4, (r, bound)
