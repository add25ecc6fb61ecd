"""Multi-node layouts on the simulated fabric (CPU): host-aware comm lanes and
hierarchical mode-1 plans.

The reference runs one node per machine over TCP (conf/config.json: 8 EC2
nodes); an MI355X deployment is several 8-GPU hosts - an xGMI mesh inside a
host, one NIC per GPU between hosts. A layer that no GPU of a host holds is
imported once per host (one slice per GPU over its NIC) and relayed inside the
host over xGMI (Node::schedule_imports), instead of crossing the network once
per GPU. The engine's comm lanes follow the same split (backend.h host_lanes).
"""

import itertools
import threading
import time

import pytest

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.models.catalog import make_workload
from distributed_llm_dissemination_amd.parallel.runtime import Runtime, layer_seed
from distributed_llm_dissemination_amd.utils.config import parse_config

MiB = 1 << 20
_keys = itertools.count()


@pytest.mark.parametrize("world,hosts", [(16, 2), (8, 2), (12, 2), (24, 3), (32, 4)])
def test_host_lanes_separate_links(world, hosts):
    """Both ends of a pair compute its lane from (src, dst) alone; every rank's
    sends and recvs sit on different lanes; inside a host every directed xGMI
    link has a lane of its own (by local index)."""
    lanes = _core.resolve_lanes(world, 0, hosts)
    assert lanes <= 32
    g = world // hosts
    for r in range(world):
        send = {d: _core.lane_of(r, d, world, lanes, hosts) for d in range(world) if d != r}
        recv = {s: _core.lane_of(s, r, world, lanes, hosts) for s in range(world) if s != r}
        assert all(0 <= l < lanes for l in list(send.values()) + list(recv.values()))
        assert not set(send.values()) & set(recv.values()), (r, send, recv)
        local = [send[d] for d in send if d // g == r // g]
        assert len(set(local)) == len(local) == g - 1


def test_one_host_lanes_unchanged():
    for world in (2, 4, 8):
        assert _core.resolve_lanes(world, 0, 1) == _core.resolve_lanes(world)
        for s in range(world):
            for d in range(world):
                if s != d:
                    assert _core.lane_of(s, d, world, _core.resolve_lanes(world), 1) == \
                        _core.lane_of(s, d, world, _core.resolve_lanes(world))


def test_config_host_field_and_uniform_hosts(monkeypatch):
    raw = {"Nodes": [{"ID": i, "Addr": "", "IsLeader": i == 0, "Host": f"m{i // 2}",
                      "InitialLayers": {"2": {str(i): {"LayerSize": MiB}}}} for i in range(4)],
           "Assignment": {str(i): {str(l): {} for l in range(4)} for i in range(4)}}
    cfg = parse_config(raw)
    assert cfg.hosts() == {0: 0, 1: 0, 2: 1, 3: 1}
    assert parse_config(cfg.to_json()).hosts() == cfg.hosts()
    rt = Runtime(cfg, 0, engine="sim", registry={0: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=f"cfg{next(_keys)}")
    try:
        assert rt.uniform_hosts() == 2
        assert rt.engine.stats().lanes == _core.resolve_lanes(4, 0, 2)
        xgmi = [(a, b, "xgmi", 1, 0) for a in range(2) for b in range(2) if a != b]
        monkeypatch.setattr(_core, "gpu_topology", lambda: xgmi, raising=False)
        bw = rt.topology_link_bw(50.0, nic_gbps=40.0)
        assert bw[(0, 1)] == bw[(3, 2)] == int(50e9)  # same host: xGMI by local device index
        assert bw[(0, 2)] == bw[(1, 3)] == int(40e9)  # across hosts: the NIC rate
    finally:
        rt.close()
    # an interleaved layout is not uniform: per-distance lanes
    for i, n in enumerate(cfg.nodes):
        n.host = f"m{i % 2}"
    rt = Runtime(cfg, 0, engine="sim", registry={0: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=f"cfg{next(_keys)}")
    try:
        assert rt.uniform_hosts() == 1
    finally:
        rt.close()


def run_hosts(n, hosts, layers, size, chunk, hierarchical, timing=None, sessions=1, adapt_links=True):
    """One cluster of n ranks on `hosts` hosts (consecutive ranks), mode 1 with
    the links policy; returns (per-session results, per-rank bytes sent to each
    peer rank, wall seconds per session)."""
    key = f"mh{next(_keys)}"
    per = n // hosts
    host_of = [i // per for i in range(n)]
    if timing is not None:
        t = _core.SimTiming()
        for k, v in timing.items():
            setattr(t, k, v)
        t.host = host_of
        _core.sim_set_timing(key, t)
    cfg = make_workload(n, layers, size, tier="host", seeding="random", chunk_bytes=chunk)
    for nd in cfg.nodes:
        nd.host = f"h{host_of[nd.id]}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=chunk, sim_key=key,
                   verify=timing is None, poison=timing is None) for i in range(n)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        out, walls = [], []
        for _ in range(sessions):
            for r in rts:
                r.prepare(1, owner_policy="links", hierarchical=hierarchical, pull_window=n - 1, adapt_links=adapt_links)
            res = [None] * n
            ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(120))) for i in range(n)]
            t0 = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            walls.append(time.perf_counter() - t0)
            assert all(x.ok for x in res), [x.error for x in res]
            out.append(res)
        if timing is None:
            for i, r in enumerate(rts):
                for l in cfg.assignment[i]:
                    assert r.layer_bytes(l) == _core.fill_random_host(size, layer_seed(0, l)), (i, l)
        sent = [r.link_stats()["sent"] for r in rts]
        holders = {l: i for i, nd in enumerate(cfg.nodes) for per_src in nd.initial_layers.values() for l in per_src}
        return out, sent, walls, host_of, holders
    finally:
        for r in rts:
            r.close()


def cross_bytes(sent, host_of):
    return sum(b for s, per in enumerate(sent) for d, b in per.items() if host_of[s] != host_of[d])


@pytest.mark.parametrize("hosts,n", [(2, 6), (3, 6)])
def test_hierarchical_import_crosses_each_host_once(hosts, n):
    """Byte-exact delivery; a layer crosses the network once per host that
    lacks it (the flat plan: once per GPU that lacks it)."""
    layers, size = 12, 4 * MiB
    _, sent, _, host_of, holders = run_hosts(n, hosts, layers, size, MiB, hierarchical=True)
    once = sum(size for l, h in holders.items() for H in set(host_of) if host_of[h] != H)
    assert cross_bytes(sent, host_of) == once
    _, sent_flat, _, _, _ = run_hosts(n, hosts, layers, size, MiB, hierarchical=False)
    per_gpu = sum(size for l, h in holders.items() for d in range(n) if host_of[d] != host_of[h])
    assert cross_bytes(sent_flat, host_of) == per_gpu == once * (n // hosts)


def test_hierarchical_plan_beats_per_gpu_imports_over_nics():
    """2 hosts x 4 GPUs, 32 layers: xGMI links and NICs at the same rate, one
    NIC per GPU shared by all of its remote peers. Importing per host needs
    1/4 of the NIC bytes of importing per GPU; the relays ride the xGMI links
    that carry the host's own layers anyway. Plans compared as planned (no
    closed-loop rates: those let the flat plan relay around its NIC-bound
    links after a session and close part of the gap)."""
    scale, slow = 1024, 8
    rate = 50e9 / scale / slow
    timing = dict(link_bps=rate, stage_bps=57.5e9 / scale / slow, nic_bps=rate, copy_bytes=False)
    kw = dict(layers=32, size=(1 << 30) // scale, chunk=(64 * MiB) // scale, timing=timing, sessions=2,
              adapt_links=False)
    _, _, hier, _, _ = run_hosts(8, 2, hierarchical=True, **kw)
    _, _, flat, _, _ = run_hosts(8, 2, hierarchical=False, **kw)
    assert min(hier) < 0.75 * min(flat), (hier, flat)


@pytest.mark.parametrize("hosts,n", [(2, 6), (3, 6), (2, 4)])
def test_mode0_broadcast_across_hosts(hosts, n):
    """Planned mode 0 (relay) on several hosts, the leader holding every layer
    (BASELINE config #2 spread over machines): scatter over the leader's host,
    each slice exported once into every other host by the GPU that holds it,
    relayed there. Byte-exact; each layer enters each other host once; the
    leader's own NIC carries nothing when its host has other GPUs."""
    key = f"mh0{next(_keys)}"
    per = n // hosts
    host_of = [i // per for i in range(n)]
    layers, size = 6, 4 * MiB
    cfg = make_workload(n, layers, size, tier="host", seeding="leader", chunk_bytes=MiB)
    for nd in cfg.nodes:
        nd.host = f"h{host_of[nd.id]}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key) for i in range(n)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for r in rts:
            r.prepare(0, relay=True)
        res = [None] * n
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(60))) for i in range(n)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert all(x.ok for x in res), [x.error for x in res]
        for i, r in enumerate(rts):
            for l in cfg.assignment[i]:
                assert r.layer_bytes(l) == _core.fill_random_host(size, layer_seed(0, l)), (i, l)
        sent = [r.link_stats()["sent"] for r in rts]
        assert cross_bytes(sent, host_of) == layers * size * (hosts - 1)
        assert sum(b for d, b in sent[0].items() if host_of[d] != host_of[0]) == 0
    finally:
        for r in rts:
            r.close()


@pytest.mark.parametrize("n,hosts", [(16, 2), (24, 3)])
def test_host_lanes_survive_rccl_round_model(n, hosts):
    """RCCL runs a group's P2P ops in rounds of one ring distance each
    (SimTiming.p2p_rounds). Hierarchical mode 1 on host-aware lanes - at 3
    hosts of 8 several remote peers share a cross-host lane - completes
    byte-exact under that model."""
    run_hosts(n, hosts, 24, 2 * MiB, MiB, hierarchical=True, timing=dict(p2p_rounds=True, copy_bytes=True, wait_s=20))


def _gather_worker(rank, world, port, fake, out):
    import os

    import torch.distributed as dist

    from distributed_llm_dissemination_amd.utils.launch import FAKE_HOSTS_ENV, gather_hosts, listen_addr

    if fake:
        os.environ[FAKE_HOSTS_ENV] = str(fake)
    else:
        os.environ.pop(FAKE_HOSTS_ENV, None)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        hosts = gather_hosts(10 + rank)
        out.put((rank, hosts, listen_addr(bool(hosts))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fake", [0, 2])
def test_gather_hosts_over_gloo(fake):
    """Under torchrun every rank learns every rank's host: one machine -> None
    (single-host plans and lanes); DISSEM_FAKE_HOSTS=2 splits 4 ranks into 2
    hosts of consecutive ranks, still listening on loopback."""
    import multiprocessing as mp
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, 4, port, fake, q)) for r in range(4)]
    for p in ps:
        p.start()
    got = dict((r, (h, a)) for r, h, a in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(4):
        hosts, addr = got[r]
        assert addr == "127.0.0.1:0"
        if fake:
            assert hosts == {10: "host0", 11: "host0", 12: "host1", 13: "host1"}
        else:
            assert hosts is None


def test_mode3_across_hosts_every_session_plans():
    """Mode 3 on 2 hosts x 4 GPUs plans with NIC budgets (LP); the closed loop
    then feeds measured link rates that span orders of magnitude next to the
    planning constants. Every session must still get a plan (the LP retries
    with other scalings of T, then falls back to the max-flow) and deliver."""
    n, hosts = 8, 2
    key = f"mh3{next(_keys)}"
    host_of = [i // 4 for i in range(n)]
    t = _core.SimTiming()
    t.host = host_of
    t.wait_s = 20
    _core.sim_set_timing(key, t)
    cfg = make_workload(n, 16, 4 * MiB, tier="host", seeding="random", chunk_bytes=MiB)
    for nd in cfg.nodes:
        nd.host = f"h{host_of[nd.id]}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key) for i in range(n)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for _ in range(3):
            for r in rts:
                r.prepare(3)
            res = [None] * n
            ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(60))) for i in range(n)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            assert all(x.ok for x in res), [x.error for x in res]
            assert res[0].flow_T > 0
            for i, r in enumerate(rts):
                for l in cfg.assignment[i]:
                    assert r.layer_bytes(l) == _core.fill_random_host(4 * MiB, layer_seed(0, l)), (i, l)
    finally:
        for r in rts:
            r.close()


@pytest.mark.parametrize("hosts,n,window", [(2, 6, 1), (3, 6, 5), (2, 8, 7)])
def test_mode2_pulls_once_per_host(hosts, n, window):
    """Mode 2 (pull / steal) on several hosts: one GPU of a host that lacks a
    layer pulls it across the network; its host peers pull it from that GPU
    once it holds it (its ack kicks it), and no job a host serves itself is
    stolen across hosts. Byte-exact, and every layer enters each other host
    exactly once (the flat pull: about once per GPU)."""
    key = f"mh2{next(_keys)}"
    per = n // hosts
    host_of = [i // per for i in range(n)]
    size = 4 * MiB
    cfg = make_workload(n, 12, size, tier="host", seeding="random", chunk_bytes=MiB)
    for nd in cfg.nodes:
        nd.host = f"h{host_of[nd.id]}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key) for i in range(n)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for r in rts:
            r.prepare(2, pull_window=window)
        res = [None] * n
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(60))) for i in range(n)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert all(x.ok for x in res), [x.error for x in res]
        for i, r in enumerate(rts):
            for l in cfg.assignment[i]:
                assert r.layer_bytes(l) == _core.fill_random_host(size, layer_seed(0, l)), (i, l)
        sent = [r.link_stats()["sent"] for r in rts]
        holders = {l: i for i, nd in enumerate(cfg.nodes) for per_src in nd.initial_layers.values() for l in per_src}
        once = sum(size for l, h in holders.items() for H in set(host_of) if host_of[h] != H)
        assert cross_bytes(sent, host_of) == once
    finally:
        for r in rts:
            r.close()
