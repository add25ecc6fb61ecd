#!/usr/bin/env python3
"""Predict T(N) of the headline bench with the planned engine on the simulated
fabric's timing model (CPU only, no payload bytes).

The schedule is the real one - leader plan, sequence numbers, lanes, groups,
staging waits - executed by the same engine code that drives RCCL; the sim
backend charges every staging copy len / PCIe and every P2P transfer
len / link on its directed link. Sizes are scaled down by --scale with the
rates scaled by the same factor, so every chunk takes its full-size time in a
fraction of the memory.

By default everything runs on the virtual clock (core/vclock.h,
parallel/simclock.py): the simulator waits in model time, so a session's
predicted length is its modeled makespan - the same number on every run and
on any host load - plus the leader's plan time measured on this CPU (the plan
is real CPU work that does not get faster with the fabric). --wall runs the
older wall-clock mode (every modeled time slept, --slowdown x slower).

    python scripts/predict_scaling.py --link-gbps 50 64 --ns 1 2 4 8
    python scripts/predict_scaling.py --ns 8 --mode0                 # BASELINE config #2
    python scripts/predict_scaling.py --ns 8 --pack fp8 --layers 126 --layer-mib 3072 --slowdown 8   # config #5
    python scripts/predict_scaling.py --ns 16 --hosts 2 --slowdown 8 [--flat]   # 2 hosts x 8 GPUs

Prints one JSON line per (link rate, N): predicted ms per step and the
aggregate GB/s value bench.py would report (N x 80 GiB / T).
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llm_dissemination_amd import _core  # noqa: E402
from distributed_llm_dissemination_amd.models.catalog import delivered_bytes, make_workload  # noqa: E402
from distributed_llm_dissemination_amd.parallel import simclock  # noqa: E402
from distributed_llm_dissemination_amd.parallel.runtime import Runtime  # noqa: E402

MiB = 1 << 20
_n = [0]
# The verify queue's device time (GB/s of checked bytes, us per launch), from
# scripts/verify_bench.py on one MI355X (profiles/r6_verify5): with peers the
# verify stream owns 32 CUs - 1.64 TB/s in 16-chunk launches, 50 us for a lone
# 64 MiB chunk; alone it has every CU - 5.69 TB/s, 23.4 us for a lone chunk.
VERIFY_MODEL = {"peers": (1640.0, 9.3), "alone": (5690.0, 11.6)}


def predict(n: int, *, layers: int = 80, layer_bytes: int = 1 << 30, chunk: int = 64 * MiB, pcie_gbps: float = 57.5,
            link_gbps: float = 50.0, scale: int = 256, mode: int = 1, lanes: int = 0, steps: int = 2,
            slow_link=None, seeding: str = "random", policy=None, plan_links: bool = False,
            slowdown: float = 1.0, tier: str = "host", pack: str = "none", plan_link_gbps=None,
            adapt_links: bool = True, disk_gbps: float = 13.3, host_share: bool = False, hosts: int = 1,
            nic_gbps: float = 50.0, host_lane_classes: int = 0, probe_mib: int = 256, warmup: int = 1,
            recv_delay=None, slow_after_probe: bool = False, virtual: bool = True,
            serialize_lanes: bool = False, trace: bool = False, verify_model: bool = True) -> dict:
    """Timed sessions of the headline workload at 1/scale size; returns the full-size prediction.

    slow_link=((s, d), frac): that directed link runs at frac of the others
    (or a list of such pairs: several slow links)
    (slow_after_probe: only from the first session on - the probe saw it at full speed).
    plan_links: the leader's plan knows every link's capacity (config Links)
    and every GPU's staging rate, at the simulated (scaled) rates: mode 1 with
    owner_policy "links" can relay around a slow link, and mode 3 plans - and
    paces its jobs at size/T - with the rates the fabric will deliver.
    plan_link_gbps: with plan_links, the rate the plan assumes for the links
    (default: the simulated one) - e.g. a constant estimate the real fabric beats.
    adapt_links: every session after the first plans on the link rates the ranks
    measured in the earlier ones (closed loop, Runtime.link_report).
    probe_mib: as bench.py, an untimed pre-flight probe of every directed link
    (this many MiB at full size, concurrent pass only) floors the closed loop's
    link capacities; 0 = no probe.
    warmup: sessions run before the `steps` timed ones (bench.py --warmup).
    recv_delay: {rank: seconds (full size)} - fault injection: that rank posts
    every receive this late (its peers' sends wait for it).
    A session's predicted time is its modeled transfer time (wall time minus
    the leader's plan, divided by `slowdown`) plus the leader's plan time at
    full weight - the plan is CPU work that does not get faster with the
    fabric. ms_per_step is the mean over the timed sessions (min_ms: the best).
    tier="disk" (BASELINE config #4): layers are files read by each rank's disk
    readers through ONE node-wide budget of disk_gbps (the node's single NVMe,
    engine/node_pacer.h), then staged over that rank's PCIe; mode 3 plans the
    ranks' disk tiers as one group.
    hosts: the N ranks sit in this many hosts (N / hosts GPUs each, an xGMI mesh
    inside a host); a transfer between hosts also occupies both GPUs' NICs at
    nic_gbps per direction (one NIC per GPU).
    slowdown: wall-clock mode only (virtual=False): run every rate this many
    times slower and divide the measured time by it (keeps the simulator's own
    per-op thread overhead small next to the modeled transfer times).
    virtual (default): model time (see the module docstring); `model_ms` lists
    each session's modeled makespan without the plan time.
    serialize_lanes: fault injection - each rank's comm lanes share one queue
    (SimTiming.serialize_lanes); the schedule tests' upper bounds must catch it.
    verify_model (default): every landed and staged chunk is CRC-checked on the
    rank's verify queue, which costs its measured device time (VERIFY_MODEL:
    the CRC walk on 32 CUs with peers, on all CUs alone); False: no checks."""
    if virtual:
        slowdown = 1.0  # model time has no simulator overhead to dilute
    plan_link_gbps = (plan_link_gbps if plan_link_gbps is not None else link_gbps) / slowdown
    level = _core.log_level()
    _core.set_log_level(3)  # per-event JSON lines on stderr would be part of the timed sessions
    try:
        with (simclock.virtual_clock() if virtual else contextlib.nullcontext()):
            return _predict(n, layers, layer_bytes, chunk, pcie_gbps, link_gbps, scale, mode, lanes, steps, slow_link,
                            seeding, policy, plan_links, slowdown, tier, pack, plan_link_gbps, adapt_links,
                            disk_gbps / slowdown, host_share, hosts, nic_gbps / slowdown, host_lane_classes, probe_mib,
                            warmup, {r: v * slowdown for r, v in (recv_delay or {}).items()}, slow_after_probe,
                            serialize_lanes, trace, verify_model)
    finally:
        _core.set_log_level(level)


def _predict(n, layers, layer_bytes, chunk, pcie_gbps, link_gbps, scale, mode, lanes, steps, slow_link, seeding,
             policy, plan_links, slowdown, tier, pack, plan_link_gbps, adapt_links, disk_gbps, host_share=False,
             hosts=1, nic_gbps=50.0, host_lane_classes=0, probe_mib=256, warmup=1, recv_delay=None,
             slow_after_probe=False, serialize_lanes=False, trace=False, verify_model=True):
    import shutil
    import tempfile

    storage = tempfile.mkdtemp(prefix="dld_predict_") if tier == "disk" else ""
    try:
        return _predict_in(n, layers, layer_bytes, chunk, pcie_gbps, link_gbps, scale, mode, lanes, steps, slow_link,
                           seeding, policy, plan_links, slowdown, tier, pack, plan_link_gbps, adapt_links, disk_gbps,
                           storage, host_share, hosts, nic_gbps, host_lane_classes, probe_mib, warmup, recv_delay,
                           slow_after_probe, serialize_lanes, trace, verify_model)
    finally:
        if storage:
            shutil.rmtree(storage, ignore_errors=True)


def _predict_in(n, layers, layer_bytes, chunk, pcie_gbps, link_gbps, scale, mode, lanes, steps, slow_link, seeding,
                policy, plan_links, slowdown, tier, pack, plan_link_gbps, adapt_links, disk_gbps, storage,
                host_share=False, hosts=1, nic_gbps=50.0, host_lane_classes=0, probe_mib=256, warmup=1,
                recv_delay=None, slow_after_probe=False, serialize_lanes=False, trace=False, verify_model=True):
    pcie_gbps, link_gbps = pcie_gbps / slowdown, link_gbps / slowdown
    key = f"predict{os.getpid()}_{_n[0]}"
    _n[0] += 1
    t = _core.SimTiming()
    t.copy_bytes = False
    t.wait_s = 600.0  # congested schedules queue transfers behind their links and NICs for long
    t.stage_bps = pcie_gbps * 1e9 / scale
    t.serialize_lanes = serialize_lanes
    t.trace = trace
    if verify_model:
        gbps, launch_us = VERIFY_MODEL["peers" if n > 1 else "alone"]
        t.verify_bps = gbps / slowdown * 1e9 / scale
        t.verify_launch_s = launch_us * 1e-6 * slowdown
    t.link_bps = link_gbps * 1e9 / scale
    slows = _slow_list(slow_link)
    slow = {(s, d): link_gbps * 1e9 / scale * frac for (s, d), frac in slows}
    if slow and not slow_after_probe:
        t.link = slow
    if recv_delay:
        t.recv_delay_s = dict(recv_delay)
    per_host = max(1, n // max(1, hosts))
    host_of = [min(i // per_host, hosts - 1) for i in range(n)]
    if hosts > 1:
        t.host = host_of
        t.nic_bps = nic_gbps * 1e9 / scale
    _core.sim_set_timing(key, t)
    lb, cb = layer_bytes // scale, chunk // scale
    cfg = make_workload(n, layers, lb, tier=tier, seeding=seeding, chunk_bytes=cb)
    if hosts > 1:
        for nd in cfg.nodes:
            nd.host = f"host{host_of[nd.id]}"
    if plan_links:
        # the plan's rates are the simulated ones (scaled): mode 3 paces jobs at size/T
        bw = int(plan_link_gbps * 1e9 / scale)
        nic_bw = int(nic_gbps * 1e9 / scale)
        cfg.links = {s: {d: (bw if host_of[s] == host_of[d] else min(bw, nic_bw)) for d in range(n) if d != s}
                     for s in range(n)}
        for (s, d), frac in slows:
            cfg.links[s][d] = int(bw * frac)
    disk = dict(storage_path=storage, node_disk_gbps=disk_gbps / scale, node_key=key) if tier == "disk" else {}
    virtual = _core.vclock_enabled()
    if virtual:
        # model time: in-process transport (no socket reader threads the clock
        # cannot count) and a barrier that waits in model time
        bar = simclock.barrier(n)
        reg = {i: f"{key}/{i}" for i in range(n)}
        rt_kw = dict(transport="inproc", registry=reg)
    else:
        bar = threading.Barrier(n).wait
        rt_kw = {}
    rts = [Runtime(cfg, i, engine="sim", chunk_bytes=cb, sim_key=key, verify=verify_model,
                   poison=False, engine_opts={"lanes": lanes, "host_lane_classes": host_lane_classes}, pack=pack,
                   host_share=host_share, barrier=bar, **(rt_kw or {"registry": {i: "127.0.0.1:0"}}), **disk)
           for i in range(n)]
    if host_share:
        for r in rts:
            r.unlink_shared()
    if not virtual:
        reg = {i: r.transport.address() for i, r in enumerate(rts)}
        for r in rts:
            r.transport.set_registry(reg)
    times, flow_Ts, plans, cached, walls, models = [], [], [], [], [], []
    flow_T = 0.0
    plan_links_used = {}
    probe_GBps = None
    try:
        if n > 1 and probe_mib > 0 and adapt_links:
            # bench.py's untimed pre-flight probe (concurrent pass): floors the link capacities
            nb = max(cb, (probe_mib << 20) // scale)
            got, _ = simclock.run_ranks([lambda r=r: r.probe_links(nb, timeout_s=600, solo=False) for r in rts])
            for r, g in zip(rts, got):
                r.observe_probe({p: v * 1e9 for p, v in g.get("concurrent", {}).items() if v},
                                {p: v * 1e9 for p, v in g.get("concurrent_in", {}).items() if v})
            conc = sorted(v for g in got for v in g.get("concurrent", {}).values() if v)
            probe_GBps = round(conc[len(conc) // 2] * scale * slowdown, 1) if conc else None
        if slow and slow_after_probe:  # the link degrades after the probe
            t.link = slow
            _core.sim_set_timing(key, t)
        for step in range(warmup + steps):
            for r in rts:
                extra = {"stage_gbps": pcie_gbps / scale} if plan_links else {}
                if plan_links and hosts > 1:
                    extra["nic_gbps"] = nic_gbps / scale
                r.prepare(mode, **{"pull_window": max(1, 2 * (n - 1)), "adapt_links": adapt_links, **extra,
                                   **(policy or {})})
            sent0 = [r.link_stats()["sent"] for r in rts]
            staged0 = [r.engine.stats().bytes_staged for r in rts]
            if trace:
                _core.sim_fabric_clear_trace(key)
            w0 = time.perf_counter()
            res, span = simclock.run_ranks([lambda r=r: r.execute(600) for r in rts])
            walls.append(time.perf_counter() - w0)
            if not all(x.ok for x in res):
                raise RuntimeError([x.error for x in res if not x.ok])
            plan_s = res[0].plan_ms / 1e3
            if virtual:
                # model time: the plan ran while the clock stood still - charge it at its CPU cost
                models.append(span)
                times.append(span + plan_s)
            else:
                times.append((span - plan_s) / slowdown + plan_s)
            plans.append(res[0].plan_ms)
            cached.append(res[0].plan_cached)
            flow_T = res[0].flow_T
            flow_Ts.append(flow_T)
            plan_links_used = rts[0].plan_link_bw()
            # bytes accounting of this session (deterministic, unlike wall time):
            # per directed link and per rank's staging, at full size
            link_bytes = {}
            for i, r in enumerate(rts):
                for p, b in r.link_stats()["sent"].items():
                    d = b - sent0[i].get(p, 0)
                    if d:
                        link_bytes[(i, p)] = d * scale
            staged = [(r.engine.stats().bytes_staged - staged0[i]) * scale for i, r in enumerate(rts)]
        lanes_used = rts[0].engine.stats().lanes
        vs = rts[0].engine.stats()
        verify_rank0 = {"calls": vs.verify_calls, "chunks": vs.verify_chunks,
                        "busy_ms_full_size": round(vs.verify_busy_ms / slowdown, 1)}
        trace_last = _core.sim_fabric_trace(key) if trace else None
        rts_est = [dict(r.link_est) for r in rts]  # per rank: the send-side busy-throughput EWMA per peer (B/s)
        rts_est_in = [dict(r.link_est_in) for r in rts]  # ... and the receive-side one per peer
    finally:
        for r in rts:
            r.close()
    timed = times[warmup:] or times
    sec = sum(timed) / len(timed)
    total = delivered_bytes(cfg) * scale
    return {"n": n, "link_GBps": link_gbps * slowdown, "pcie_GBps": pcie_gbps * slowdown, "mode": mode, "tier": tier,
            **({"node_disk_GBps": disk_gbps * slowdown} if tier == "disk" else {}),
            **({"pack": pack, "layers": layers, "layer_MiB": layer_bytes >> 20} if pack != "none" else {}),
            **({"hosts": hosts, "nic_GBps": nic_gbps * slowdown} if hosts > 1 else {}),
            "seeding": seeding, **({"policy": policy} if policy else {}), **({"host_share": True} if host_share else {}),
            "lanes": lanes_used, "ms_per_step": round(sec * 1e3, 1), "min_ms": round(min(timed) * 1e3, 1),
            "warmup": warmup, "times_ms": [round(x * 1e3, 1) for x in times],
            **({"clock": "virtual", "model_ms": [round(x * 1e3, 3) for x in models],
                "model_ms_per_step": round(sum(models[warmup:] or models) / len(models[warmup:] or models) * 1e3, 3),
                "wall_s": round(sum(walls), 2)} if virtual else {"clock": "wall"}),
            "plan_ms": [round(x, 2) for x in plans], "plan_cached": cached,
            **({"probe_GBps": probe_GBps} if probe_GBps else {}),
            **({"flow_T_ms": [round(x / slowdown * 1e3, 1) for x in flow_Ts]} if any(flow_Ts) else {}),
            **({"plan_link_GBps_last": {f"{a}->{b}": round(v * scale * slowdown / 1e9, 1)
                                        for (a, b), v in sorted(plan_links_used.items())}} if plan_links_used else {}),
            "busy_GBps": {f"{i}->{p}": round(v * scale * slowdown / 1e9, 1) for i, r in enumerate(rts_est)
                          for p, v in sorted(r.items())},
            "busy_in_GBps": {f"{p}->{i}": round(v * scale * slowdown / 1e9, 1) for i, r in enumerate(rts_est_in)
                             for p, v in sorted(r.items())},
            "link_GiB_last": {f"{a}->{b}": round(v / 2**30, 3) for (a, b), v in sorted(link_bytes.items())},
            "staged_GiB_last": [round(v / 2**30, 3) for v in staged],
            "modeled_ms_last": round(modeled_ms(link_bytes, staged, n, link_gbps * slowdown, pcie_gbps * slowdown,
                                                 slow_link) * 1e3, 1),
            "value_GBps": round(total / sec / 1e9, 1), "scale": scale,
            **({"trace_last": trace_last} if trace else {}),
            **({"verify_rank0_all_sessions": verify_rank0} if verify_model else {}),
            **({"planned_T_ms": round(flow_T * 1e3 / slowdown, 1)} if flow_T > 0 else {})}


def closed_form_ms(n: int, *, layers: int = 80, layer_bytes: int = 1 << 30, link_gbps: float = 50.0,
                   pcie_gbps: float = 57.5, tier: str = "host", disk_gbps: float = 13.3, mode0: bool = False) -> float:
    """The physical lower bound of one step, in ms.

    Modes 1-3, random seeding (the headline): every GPU stages its 1/N of the
    layers over its PCIe and receives 1/N from each peer over that link, both
    overlapped: total / N / min(PCIe, link) (N = 1: total / PCIe); from the
    node's one NVMe (tier "disk") at least total / NVMe.
    Mode 0 (config #2, the leader holds every layer): each receiver takes
    every byte in over its N - 1 links, total / (N - 1) / link; from host
    memory (tier "host") the leader's PCIe carries every byte too."""
    total = layers * layer_bytes
    if mode0:
        if n < 2:
            return 0.0
        t = total / (n - 1) / (link_gbps * 1e9)
        if tier == "host":
            t = max(t, total / (pcie_gbps * 1e9))
        return t * 1e3
    t = total / n / min(pcie_gbps * 1e9, link_gbps * 1e9 if n > 1 else float("inf"))
    if tier == "disk":
        t = max(t, total / (disk_gbps * 1e9))
    return t * 1e3


def _slow_list(slow_link):
    """slow_link as a list of ((s, d), frac)."""
    if not slow_link:
        return []
    return [slow_link] if isinstance(slow_link[0][0], int) else list(slow_link)


def modeled_ms(link_bytes, staged, n, link_gbps, pcie_gbps, slow_link=None) -> float:
    """A load-independent lower bound of a session from its bytes accounting:
    the busiest directed link's bytes / its rate, or the busiest rank's staged
    bytes / PCIe, whichever is longer (seconds; the wall clock of the
    simulated threads does not enter it)."""
    t = 0.0
    for (s, d), b in link_bytes.items():
        rate = link_gbps * 1e9 * dict((tuple(k), f) for k, f in _slow_list(slow_link)).get((s, d), 1.0)
        t = max(t, b / rate)
    for b in staged:
        t = max(t, b / (pcie_gbps * 1e9))
    return t


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ns", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--link-gbps", type=float, nargs="+", default=[50.0])
    ap.add_argument("--pcie-gbps", type=float, default=57.5)
    ap.add_argument("--scale", type=int, default=1024)
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--slowdown", type=float, default=4.0, help="--wall only: rates this many times slower")
    ap.add_argument("--wall", action="store_true",
                    help="the wall-clock simulator (sleeps every modeled time) instead of model time")
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--layer-mib", type=int, default=1024)
    ap.add_argument("--tier", choices=["host", "disk"], default="host",
                    help="disk: BASELINE config #4 - layer files behind one node-wide NVMe budget (--disk-gbps)")
    ap.add_argument("--disk-gbps", type=float, default=13.3, help="the node's NVMe read rate (profiles/r1_diskspeed.log)")
    ap.add_argument("--pack", choices=["none", "fp8"], default="none",
                    help="fp8: BASELINE config #5 (bf16 over PCIe, packed fp8 over the links)")
    ap.add_argument("--host-share", action="store_true",
                    help="with --mode0: the leader's host layers in node-shared memory, one slice staged per rank")
    ap.add_argument("--hosts", type=int, default=1,
                    help="the N ranks on this many hosts (one NIC per GPU at --nic-gbps between hosts)")
    ap.add_argument("--nic-gbps", type=float, default=50.0)
    ap.add_argument("--flat", action="store_true",
                    help="with --hosts: every dest imports from the holders itself (no per-host import + relay)")
    ap.add_argument("--mode0", action="store_true",
                    help="BASELINE config #2 instead: mode 0 from the leader (relay vs ncclBroadcast, host vs HBM source)")
    ap.add_argument("--steps", type=int, default=4, help="timed sessions (mean reported)")
    ap.add_argument("--warmup", type=int, default=1, help="untimed sessions first (bench.py --warmup)")
    ap.add_argument("--probe-mib", type=int, default=256, help="pre-flight link probe at full size, as bench.py (0: none)")
    ap.add_argument("--owner-policy", default="links", choices=["random", "balanced", "links"],
                    help="mode 1's owner choice (bench.py's default: links)")
    ap.add_argument("--pull-window", type=int, default=0,
                    help="mode 2: jobs in flight per sender (0: 2 (N - 1), as bench.py)")
    args = ap.parse_args()
    common = dict(steps=args.steps, warmup=args.warmup, probe_mib=args.probe_mib, virtual=not args.wall)
    _core.set_log_level(3)
    if args.mode0:
        for lg in args.link_gbps:
            for n in args.ns:
                if args.host_share:
                    r = predict(n, link_gbps=lg, pcie_gbps=args.pcie_gbps, scale=args.scale, lanes=args.lanes,
                                mode=0, slowdown=args.slowdown, seeding="leader", tier="host", host_share=True, **common)
                    print(json.dumps(r), flush=True)
                    continue
                for tier in ("device", "host"):
                    for relay, coll in ((True, False), (False, True)):
                        r = predict(n, link_gbps=lg, pcie_gbps=args.pcie_gbps, scale=args.scale, lanes=args.lanes,
                                    mode=0, slowdown=args.slowdown, seeding="leader", tier=tier,
                                    policy={"relay": relay, "collective": coll, "hierarchical": not args.flat},
                                    hosts=args.hosts, nic_gbps=args.nic_gbps, **common)
                        if args.hosts == 1:
                            r["closed_form_ms"] = round(closed_form_ms(n, link_gbps=lg, pcie_gbps=args.pcie_gbps,
                                                                       tier=tier, mode0=True), 1)
                        print(json.dumps(r), flush=True)
        return 0
    for lg in args.link_gbps:
        for n in args.ns:
            r = predict(n, link_gbps=lg, pcie_gbps=args.pcie_gbps, scale=args.scale, lanes=args.lanes, mode=args.mode,
                        slowdown=args.slowdown, layers=args.layers, layer_bytes=args.layer_mib << 20, pack=args.pack,
                        tier=args.tier, disk_gbps=args.disk_gbps, hosts=args.hosts, nic_gbps=args.nic_gbps,
                        policy={"owner_policy": args.owner_policy, "hierarchical": not args.flat,
                                **({"pull_window": args.pull_window} if args.pull_window else {})}, **common)
            # closed form: every GPU stages 80/N GiB over PCIe and gets
            # 80/N GiB from each peer over its link; both overlap
            if args.pack == "none" and args.hosts == 1:
                r["closed_form_ms"] = round(closed_form_ms(n, layers=args.layers, layer_bytes=args.layer_mib << 20,
                                                           link_gbps=lg, pcie_gbps=args.pcie_gbps, tier=args.tier,
                                                           disk_gbps=args.disk_gbps), 1)
            print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
