"""Schedules under the simulated fabric's timing and RCCL models, in model time.

SimTiming gives the sim fabric per-link bandwidth, per-rank staging (PCIe)
bandwidth and, optionally, RCCL's round-by-round P2P execution. These tests
check what the byte-exact tests in test_planned_sim.py cannot: that lanes keep
irregular groups safe under RCCL's round model, that token-bucket pacing holds
configured rates (reference writeWithLimit, transport.go:407-424; mode-3
size/T rates, node.go:1281; tier LimitRate on self loads, node.go:1615-1624),
and how close the headline schedule's T(N) comes to its physical bound.

Every session here runs on the virtual clock (csrc/core/vclock.h,
parallel/simclock.py): the simulator's threads wait in model time and the
clock jumps to the next modeled event once every one of them is blocked, so
a session's length is the schedule's modeled makespan - identical on every
run, on an idle or a loaded host. That is what lets every timing assertion
below take BOTH bounds: no faster than the bytes allow (the bound) and no
slower than a few percent above it (the schedule's efficiency). A change that
serialized the comm lanes or left links idle fails here
(test_upper_bounds_catch_serialized_lanes proves the bounds have teeth).
Reference schedules judged: node.go:554-608 (mode 1), flow.go:146-219
(mode 3), node.go:741-807 / :909-1073 (mode 2), node.go:326-352 (mode 0).
"""

import itertools
import os
import sys
import threading
import time

import pytest

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.models.catalog import make_workload
from distributed_llm_dissemination_amd.parallel import simclock
from distributed_llm_dissemination_amd.parallel.runtime import Runtime

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import predict_scaling  # noqa: E402

MiB = 1 << 20
_keys = itertools.count()
HEADLINE = dict(scale=1024, link_gbps=50.0, pcie_gbps=57.5, policy={"owner_policy": "links"})


def run_timed(cfg, mode, timing=None, lanes=0, chunk=MiB, verify=True, sessions=1, runtime_kw=None, **policy):
    """Sessions of `cfg` on the sim fabric in model time; returns (seconds of the last, results)."""
    key = f"tsim{os.getpid()}_{next(_keys)}"
    if timing is not None:
        _core.sim_set_timing(key, timing)
    n = len(cfg.nodes)
    with simclock.virtual_clock():
        reg = {i: f"{key}/{i}" for i in range(n)}
        rts = [Runtime(cfg, i, engine="sim", transport="inproc", registry=reg, chunk_bytes=chunk, sim_key=key,
                       verify=verify, engine_opts={"lanes": lanes}, **(runtime_kw or {})) for i in range(n)]
        try:
            for _ in range(sessions):
                for r in rts:
                    r.prepare(mode, **policy)
                res, dt = simclock.run_ranks([lambda r=r: r.execute(60) for r in rts])
                assert all(x.ok for x in res), [x.error for x in res]
            return dt, res
        finally:
            for r in rts:
                r.close()


def test_model_time_is_deterministic():
    """Two runs of the same N = 4 prediction give the same modeled makespan
    to the microsecond, session for session (the plan time, real CPU work,
    is reported beside it and not part of it)."""
    a = predict_scaling.predict(4, steps=2, **HEADLINE)
    b = predict_scaling.predict(4, steps=2, **HEADLINE)
    assert a["clock"] == "virtual" and a["model_ms"] == b["model_ms"], (a["model_ms"], b["model_ms"])


def test_lanes_keep_irregular_groups_safe_under_rccl_rounds():
    """Mode 2 at 8 ranks dispatches jobs as acks return, so ranks form
    different groups. Under RCCL's round model (a group's ops run one ring
    distance at a time) a multi-distance group can wait on itself across ranks
    - the 8-rank hang first seen on the GPU box with one lane. With world-1
    lanes every group holds one distance and the session completes."""
    cfg = make_workload(8, 16, 4 * MiB, tier="host", seeding="random", chunk_bytes=MiB)
    t = _core.SimTiming()
    t.p2p_rounds = True
    _, res = run_timed(cfg, 2, t, lanes=0, sessions=2, pull_window=2)
    assert res[0].engine_stats["verify_failures"] == 0


def test_tier_rate_paces_staging():
    """A host tier with a LimitRate (config Sources) is staged at exactly that
    rate: 8 x 1 MiB at 40 MB/s. The bucket's burst of one chunk goes at once
    (x/time/rate's initial burst), so the last chunk starts after 7 MiB of
    tokens: the session takes 7 MiB / rate, within the engine's 20 us poll."""
    rate = 40_000_000
    cfg = make_workload(1, 4, 2 * MiB, tier="host", tier_rate=rate, chunk_bytes=MiB)
    dt, res = run_timed(cfg, 1)
    want = 7 * MiB / rate
    assert want <= dt <= want * 1.01, (dt, want)
    assert res[0].engine_stats["paced"] > 0


def test_mode3_jobs_finish_at_the_planned_T():
    """Mode 3 paces every job at size/T (node.go:1281): with the leader's 50 MB/s
    NetworkBW as the binding cut, T is the closed form. A job is 8 chunks and
    its bucket's burst is two, so it cannot end before 6/8 T, and a schedule
    that keeps to the plan ends by T (plus 5 %)."""
    cfg = make_workload(4, 4, 2 * MiB, tier="host", seeding="leader", network_bw=50_000_000, chunk_bytes=MiB // 4)
    dt, res = run_timed(cfg, 3, chunk=MiB // 4)
    T = res[0].flow_T
    assert T == pytest.approx(3 * 4 * 2 * MiB / 50e6, rel=0.02)
    assert T * 6 / 8 <= dt <= 1.05 * T, (dt, T)
    assert res[0].engine_stats["paced"] > 0


def test_mode3_hbm_ingress_budget_binds_the_plan():
    """The mode-3 graph's per-GPU HBM ingress cap (prepare(hbm_gbps=...),
    SURVEY C13'): with every dest's ingress at 20 MB/s and no other limit,
    T is the busiest dest's bytes / 20 MB/s, and the paced jobs end between
    6/8 T (two chunks of burst) and 1.05 T."""
    cfg = make_workload(3, 3, 2 * MiB, tier="host", seeding="leader", chunk_bytes=MiB // 4)
    dt, res = run_timed(cfg, 3, chunk=MiB // 4, hbm_gbps=0.02)
    T = res[0].flow_T
    assert T == pytest.approx(3 * 2 * MiB / 20e6, rel=0.02)
    assert T * 6 / 8 <= dt <= 1.05 * T, (dt, T)


@pytest.mark.parametrize("n", [1, 2, 4, 8])
@pytest.mark.parametrize("mode", [1, 3])
def test_headline_schedule_within_3pct_of_the_link_bound(mode, n):
    """The headline schedule (80 x 1 GiB, random seeding, at 1/1024 size with
    rates scaled alike): every GPU stages exactly 80/N GiB over PCIe and every
    directed link carries exactly 80/N GiB, so the step cannot beat
    85.9 GB / (N * min(PCIe, link)); modes 1 and 3 stay within 3 % of it in
    model time, every session (the warm-up one too). Measured: +0.14 / 0.28 /
    0.56 % at N = 2 / 4 / 8 - one chunk's staging before the first transfer."""
    r = predict_scaling.predict(n, mode=mode, steps=1, **HEADLINE)
    bound = predict_scaling.closed_form_ms(n)
    assert r["staged_GiB_last"] == [pytest.approx(80 / n, rel=1e-3)] * n, r
    assert len(r["link_GiB_last"]) == n * (n - 1), r
    assert all(v == pytest.approx(80 / n, rel=1e-3) for v in r["link_GiB_last"].values()), r
    for ms in r["model_ms"]:
        assert bound * 0.999 <= ms <= bound * 1.03, (n, mode, r["model_ms"], bound)
    if mode == 3 and n > 1:
        assert r["planned_T_ms"] == pytest.approx(bound, rel=1e-3), r


@pytest.mark.parametrize("n", [2, 4, 8])
def test_mode0_relay_within_3pct_of_ingress_bound(n):
    """BASELINE config #2: the leader holds all 80 layers in HBM; the relay
    broadcast scatters 1/(N-1) of each layer and every receiver relays its
    slice to the others, so each receiver's N - 1 ingress links carry every
    byte: T >= 85.9 GB / (N - 1) / link. The schedule stays within 3 %
    (measured +0.0 / 0.31 / 0.63 % at N = 2 / 4 / 8)."""
    r = predict_scaling.predict(n, mode=0, steps=1, seeding="leader", tier="device",
                                policy={"relay": True, "collective": False}, **{k: v for k, v in HEADLINE.items()
                                                                               if k != "policy"})
    bound = predict_scaling.closed_form_ms(n, tier="device", mode0=True)
    for ms in r["model_ms"]:
        assert bound * 0.999 <= ms <= bound * 1.03, (n, r["model_ms"], bound)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_mode2_pull_schedule_within_3pct_of_the_bound(n):
    """Mode 2 (pull / steal, node.go:741-807, :909-1073) on the headline
    workload: jobs are dispatched as acks return, yet it stays within 3 % of
    the same bound (measured +0.39 / 0.28 / 0.56 % at N = 2 / 4 / 8), every
    session. Two things keep its links fed (scripts/sim_timeline.py showed
    the idle stretches): pull batches are job-major on the lanes
    (Message.order), and a rank's loads of its own layers never queue whole
    layers on its copy queue ahead of the chunks its sends wait for
    (PlannedEngine kPromoteAhead). Before: 224-241 ms at N = 8."""
    r = predict_scaling.predict(n, mode=2, steps=1, **HEADLINE)
    bound = predict_scaling.closed_form_ms(n)
    for ms in r["model_ms"]:
        assert bound * 0.999 <= ms <= bound * 1.03, (n, r["model_ms"], bound)


def test_upper_bounds_catch_serialized_lanes():
    """The bounds above have teeth: with every rank's comm lanes forced onto
    one queue (SimTiming.serialize_lanes - as if the 14 lanes of N = 8 were
    one stream) the same schedule misses the 3 % bound by far (32 layers: the
    serialized schedule is slow to simulate, not only to run)."""
    bound = predict_scaling.closed_form_ms(8, layers=32)
    r = predict_scaling.predict(8, layers=32, mode=1, steps=1, warmup=0, serialize_lanes=True, **HEADLINE)
    assert min(r["model_ms"]) > 1.5 * bound, (r["model_ms"], bound)


def _max_link_time(r, slow=None, frac=1.0, gbps=50.0):
    """Seconds the busiest directed link needs for the last session's bytes."""
    t = 0.0
    for k, gib in r["link_GiB_last"].items():
        rate = gbps * 1e9 * (frac if k == slow else 1.0)
        t = max(t, gib * 2**30 / rate)
    return t


def test_slow_link_costs_at_most_a_seventh_with_the_link_aware_plan():
    """One directed link at half speed (8 ranks, headline mode 1, 1/1024 size).
    Lanes are per directed link, so the slow link holds back only its own
    transfers; the leader's link-aware plan (owner policy "links" with the
    config's Links) moves chunk slices of the layers it carries onto relays -
    ranks that receive the same layer directly - until the slowest link no
    longer sets the pace: its bytes shrink to about half, the busiest link's
    time is within 1/7 of the uniform plan's, and so is the session's model
    time; a plan that ignores the link needs ~2x."""
    kw = dict(layers=32, mode=1, steps=1, adapt_links=False, **HEADLINE)
    base = predict_scaling.predict(8, **kw)
    blind = predict_scaling.predict(8, slow_link=((0, 1), 0.5), **kw)
    planned = predict_scaling.predict(8, slow_link=((0, 1), 0.5), plan_links=True, **kw)
    t_base = _max_link_time(base)
    assert _max_link_time(blind, "0->1", 0.5) > 1.9 * t_base, (base, blind)
    assert _max_link_time(planned, "0->1", 0.5) <= t_base * (1 + 1 / 7), (base, planned)
    others = sorted(v for k, v in planned["link_GiB_last"].items() if k != "0->1")
    assert planned["link_GiB_last"]["0->1"] <= 0.6 * others[len(others) // 2], planned
    assert max(blind["model_ms"]) > 1.8 * max(base["model_ms"]), (base["model_ms"], blind["model_ms"])
    assert max(planned["model_ms"]) <= max(base["model_ms"]) * (1 + 1 / 7) * 1.03, (base["model_ms"],
                                                                                   planned["model_ms"])


def test_client_stream_cut_through_to_peers():
    """C17 pipe at chunk grain on the GPU data plane: node 1's external client
    streams layer 9 at 20 MB/s; nodes 0 and 2 need it from node 1. Node 1
    stages and forwards each chunk as soon as it has landed in host memory
    (transport.go:144-196 tees the TCP stream the same way): node 0 holds
    bytes of the layer from node 1 while node 1's stream is still arriving
    (store-and-forward would start only after it), and every byte arrives.
    (Wall clock: the client streams over a real TCP socket.)"""
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
    overlap = []  # (stream bytes node 1 had, bytes node 0 had from node 1) while the stream ran
    stop = threading.Event()

    def watch():
        s0 = rts[1].transport.bytes_received
        while not stop.is_set():
            got = rts[1].transport.bytes_received - s0
            fwd = rts[0].engine.stats().peer_recv.get(1, 0)
            if 0 < fwd and got < size:
                overlap.append((got, fwd))
            time.sleep(0.002)

    try:
        for r in rts:
            r.prepare(1)
        w = threading.Thread(target=watch)
        w.start()
        res, _ = simclock.run_ranks([lambda r=r: r.execute(60) for r in rts])
        stop.set()
        w.join()
        assert all(x.ok for x in res), [x.error for x in res]
        for r in rts:
            assert r.layer_bytes(9) == data
        assert overlap, "node 0 got nothing from node 1 before node 1's stream ended (store-and-forward)"
    finally:
        stop.set()
        for r in rts:
            r.close()
        client.stop()
        ct.close()


def test_closed_loop_routes_around_an_unconfigured_slow_link():
    """Closed-loop link rates (Runtime.link_report): one directed link runs at
    half speed and NOTHING in the config or the plan says so. The pre-flight
    probe reads it slow (one observation), the first session's busy throughput
    again (two in a row): from the second session on the leader plans on its
    measured rate and relays around it, so the link carries about half the
    bytes and the busiest link's time is back within 1/7 of a uniform mesh's
    (reference analog: node.go:774-793 times jobs, :1044-1053 steers by them)."""
    kw = dict(layers=32, mode=1, probe_mib=1024, **HEADLINE)
    r = predict_scaling.predict(8, slow_link=((0, 1), 0.5), steps=1, warmup=1, **kw)
    plan = r["plan_link_GBps_last"]
    assert plan["0->1"] == pytest.approx(25.0, abs=0.5) and plan["1->0"] == pytest.approx(50.0, abs=0.5), plan
    uniform = 32 / 8 * 2**30 / 50e9  # a uniform mesh's busiest link, 4 GiB at 50 GB/s
    assert _max_link_time(r, "0->1", 0.5) <= uniform * (1 + 1 / 7), r
    assert r["model_ms"][-1] <= uniform * 1e3 * (1 + 1 / 7) * 1.03, r["model_ms"]
    others = sorted(v for k, v in r["link_GiB_last"].items() if k != "0->1")
    assert r["link_GiB_last"]["0->1"] <= 0.6 * others[len(others) // 2], r


@pytest.mark.parametrize("mode", [1, 3])
def test_closed_loop_keeps_a_uniform_mesh_uniform(mode):
    """On a uniform 50 GB/s mesh the closed loop must be harmless: the leader
    plans every link at exactly 50.0 GB/s (each link is timed at both ends and
    planned on the faster reading: the later poster times the transfer alone),
    the plan moves exactly the bytes per link of the plan that knows the
    fabric, and it does not change from one session to the next (the leader
    replays it from the plan cache)."""
    kw = dict(mode=mode, steps=3, warmup=1, **HEADLINE)
    fixed = predict_scaling.predict(8, plan_links=True, adapt_links=False, **kw)
    adapt = predict_scaling.predict(8, probe_mib=4096, **kw)
    rates = set(adapt["plan_link_GBps_last"].values())
    assert rates == {50.0}, adapt["plan_link_GBps_last"]
    assert adapt["link_GiB_last"] == fixed["link_GiB_last"], (adapt, fixed)
    assert all(adapt["plan_cached"][2:]), adapt  # the same plan session after session
    assert adapt["model_ms"][1:] == fixed["model_ms"][1:], (adapt["model_ms"], fixed["model_ms"])
    if mode == 3:
        assert adapt["flow_T_ms"][-1] == pytest.approx(fixed["flow_T_ms"][-1], rel=1e-3), (adapt, fixed)


def test_closed_loop_sees_a_link_that_slows_after_the_probe():
    """The pre-flight probe saw every link at 50 GB/s; then link 0->1 drops to
    half. The probe floors a link's capacity only until sessions have measured
    it (Runtime.LINK_PROBE_SESSIONS), so after two sessions at half speed the
    leader plans 0->1 at its measured rate and moves bytes off it."""
    kw = dict(layers=32, mode=1, probe_mib=1024, **HEADLINE)
    r = predict_scaling.predict(8, slow_link=((0, 1), 0.5), steps=3, warmup=1, slow_after_probe=True, **kw)
    plan = r["plan_link_GBps_last"]
    assert plan["0->1"] == pytest.approx(25.0, abs=0.5) and plan["1->0"] == pytest.approx(50.0, abs=0.5), plan
    assert r["busy_GBps"]["0->1"] == pytest.approx(25.0, abs=0.5), r["busy_GBps"]  # timed at the sending end
    assert r["busy_in_GBps"]["0->1"] == pytest.approx(25.0, abs=0.5), r["busy_in_GBps"]  # ... and the receiving one
    others = sorted(v for k, v in r["link_GiB_last"].items() if k != "0->1")
    assert r["link_GiB_last"]["0->1"] <= 0.6 * others[len(others) // 2], r


def test_late_receiver_does_not_lower_link_estimates():
    """A rank that posts its receives late (every P2P group holding a recv, 2 ms
    at full size) makes its peers' sends wait: their busy throughput towards it
    reads low. That is not a slow link - the closed loop must not plan it as
    one: every link into the late rank stays at the probe's level, and the
    plan stays uniform."""
    kw = dict(layers=16, mode=1, steps=2, warmup=1, probe_mib=1024, **HEADLINE)
    r = predict_scaling.predict(4, recv_delay={2: 0.002}, **kw)
    busy = r["busy_GBps"]
    into = [v for k, v in busy.items() if k.endswith("->2")]
    other = [v for k, v in busy.items() if not k.endswith("->2")]
    assert max(into) < min(other), busy  # the injection did slow the sends into rank 2
    # ... as timed at the sending end; the receiving end timed them alone
    assert all(v == pytest.approx(50.0, abs=0.5) for k, v in r["busy_in_GBps"].items() if k.endswith("->2"))
    plan = r["plan_link_GBps_last"]
    assert set(plan.values()) == {50.0}, plan


def test_mode3_plans_at_the_probed_rate_not_the_constant():
    """Mode 3 plans T - and paces every job at size/T (node.go:1281) - from its
    link rates. The planning constant says 40 GB/s while the fabric delivers 56
    (1.4x): paced transfers never reveal spare capacity in their busy
    throughput, so the closed loop takes its capacities from the pre-flight
    probe. Already the first session plans on the probed rate: T is the
    56 GB/s closed form, not the 40 GB/s one, and every session ends within
    5 % of its planned T."""
    kw = dict(layers=16, scale=1024, link_gbps=56.0, plan_link_gbps=40.0, pcie_gbps=200.0, mode=3, steps=2,
              plan_links=True)
    blind = predict_scaling.predict(4, adapt_links=False, **kw)
    probed = predict_scaling.predict(4, probe_mib=1024, **kw)
    assert all(T == pytest.approx(blind["flow_T_ms"][0], rel=1e-3) for T in blind["flow_T_ms"]), blind
    for T, ms in zip(probed["flow_T_ms"], probed["model_ms"]):
        assert T <= blind["flow_T_ms"][0] * 40 / 56 * 1.05, (probed, blind)
        assert ms <= T * 1.05, (probed["model_ms"], probed["flow_T_ms"])


def test_node_shared_disk_budget_paces_every_rank(tmp_path):
    """One NVMe per node (config #4 at N > 1): the ranks' disk readers draw from
    one node-wide budget (engine/node_pacer.h): 4 ranks loading 8 x 1 MiB at a
    20 MB/s node rate take the node's 8 MiB / 20 MB/s, not 1/4 of it, and
    (links and staging unmodeled here) not more than 5 % beyond it."""
    cfg = make_workload(4, 8, MiB, tier="disk", seeding="random", chunk_bytes=MiB // 4)
    key = f"disk{os.getpid()}_{next(_keys)}"
    dt, res = run_timed(cfg, 1, chunk=MiB // 4,
                        runtime_kw=dict(storage_path=str(tmp_path), node_disk_gbps=0.02, node_key=key))
    want = 8 * MiB / 20e6
    assert want * 0.99 <= dt <= want * 1.05, (dt, want)
    assert sum(x.engine_stats["disk_wait_ms"] for x in res) > 0


def test_predicted_disk_tier_is_bound_by_the_node_nvme():
    """predict_scaling --tier disk: at N = 4 the headline workload from NVMe is
    bound by the node's single device (16 GiB / 13.3 GB/s here), not by
    N x per-GPU staging: every layer byte is staged exactly once somewhere and
    the step takes the NVMe time, within 5 %."""
    r = predict_scaling.predict(4, scale=4096, steps=1, tier="disk", layers=16)
    bound = 16 * (1 << 30) / 13.3e9
    assert sum(r["staged_GiB_last"]) == pytest.approx(16, rel=1e-3), r
    for ms in r["model_ms"]:
        assert bound * 0.99 <= ms / 1e3 <= bound * 1.05, (r["model_ms"], bound)


def test_closed_loop_plans_a_node_with_slow_egress_on_every_link():
    """node 0's egress runs at half speed on EVERY link. Node 0
    reports one level for all its links - its own median, low - while each
    receiver reports the link at its uniform (fast) level until it has
    flagged it over two observations. Taking the faster of the two ends, as
    for a late receiver, would hide the slow egress; a node whose level lies
    below 0.7 of the median level is planned on the slower reading
    (Node::merged_link_rates), so already the first session plans node 0's
    links at their measured 25 GB/s and moves bytes off them."""
    slow = [((0, d), 0.5) for d in range(1, 8)]
    kw = dict(layers=32, mode=1, probe_mib=1024, **HEADLINE)
    r = predict_scaling.predict(8, slow_link=slow, steps=1, warmup=0, **kw)
    plan = r["plan_link_GBps_last"]
    assert all(plan[f"0->{d}"] == pytest.approx(25.0, abs=0.5) for d in range(1, 8)), plan
    assert all(plan[f"{s}->{d}"] == pytest.approx(50.0, abs=0.5) for s in range(1, 8) for d in range(8) if d != s), plan
    blind = predict_scaling.predict(8, slow_link=slow, steps=1, warmup=0, adapt_links=False, **kw)
    assert max(r["model_ms"]) < 0.8 * max(blind["model_ms"]), (r["model_ms"], blind["model_ms"])
