"""CLI with the reference's flags (cmd/main.go:15-220).

    python -m distributed_llm_dissemination_amd -id 0 -f conf/config.json -m 1 [-s DIR] [-l] [-c] [-v]

One process per node. With ``--engine rccl`` the processes are GPU ranks
launched by torchrun (``-id`` defaults to the node at position RANK in the
sorted node ids) and layers move over RCCL/xGMI into HBM; with the default
``--engine host`` layers move over TCP into host memory, as in the reference.
Stdout contract kept: ``launching leader...`` / ``launching receiver...`` banners
and ``Time to deliver: <Go duration>``.
"""

from __future__ import annotations

import argparse
import datetime
import hashlib
import json
import os
import signal
import sys
import time

USAGE = "usage: -id 0 -f config.json -s . -m 2 -l -v"


def go_duration(seconds: float) -> str:
    """time.Duration.String() formatting (e.g. 59.87s, 1m2.5s, 150.2ms, 12µs)."""
    ns = int(round(seconds * 1e9))
    if ns == 0:
        return "0s"
    neg = ns < 0
    ns = abs(ns)

    def trim(v: float) -> str:
        s = f"{v:.9f}".rstrip("0").rstrip(".")
        return s

    if ns < 1000:
        out = f"{ns}ns"
    elif ns < 1_000_000:
        out = trim(ns / 1e3) + "µs"
    elif ns < 1_000_000_000:
        out = trim(ns / 1e6) + "ms"
    else:
        h, rem = divmod(ns, 3600 * 10**9)
        m, rem = divmod(rem, 60 * 10**9)
        s = trim(rem / 1e9) + "s"
        out = (f"{h}h" if h else "") + (f"{m}m" if (h or m) else "") + s
    return ("-" if neg else "") + out


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="distributor", add_help=True)
    p.add_argument("-id", type=int, default=None, help="my ID")
    p.add_argument("-f", default="", help="filename of topology JSON file")
    p.add_argument("-s", default="", help="path of storing layers")
    p.add_argument("-m", type=int, default=-1, help="0: naive, 1: layer retransmit, 2: pull, 3: flow")
    p.add_argument("-l", action="store_true", help="create layer files and exit")
    p.add_argument("-c", action="store_true", help="if the process is client")
    p.add_argument("-v", action="store_true", help="output debug messages")
    # extensions
    p.add_argument("--engine", default="auto", choices=["auto", "host", "rccl"],
                   help="data plane: host (TCP into RAM, the reference) or rccl (RCCL/xGMI into HBM); "
                        "auto = rccl under torchrun with a GPU visible, else host")
    p.add_argument("--chunk-mib", type=int, default=64)
    p.add_argument("--pack", default="none", choices=["none", "fp8"],
                   help="fp8: bf16 layers are packed to block-scaled e4m3fn on staging (wire + HBM format)")
    p.add_argument("--store", default="packed", choices=["packed", "bf16"],
                   help="with --pack fp8: bf16 = also keep each layer dequantized to bf16 in HBM (fused "
                        "verify+unpack kernel on every landed chunk)")
    p.add_argument("--verify", default="crc32c", choices=["none", "crc32c"])
    p.add_argument("--weights", default="", metavar="PRESET",
                   help="layers hold random-init decoder-layer weights of this model (models/weights.py presets: "
                        "tiny, llama3-8b, llama3-70b, llama3.1-405b; LayerSize must equal the preset's layer "
                        "bytes) instead of random bytes; after delivery each rank runs its layers' forward pass "
                        "on the received parameters")
    p.add_argument("--verify-cus", type=int, default=-1,
                   help="rccl: the verify stream runs on the last N CUs only, RCCL lanes and copies on the others "
                        "(-1: 32 - CUs 28-31 of each XCD - with peers, 128 with --store bf16, 0 alone; 0: shared)")
    p.add_argument("--lanes", type=int, default=0,
                   help="rccl: independent comm lanes (RCCL communicator + HIP stream + dedicated HW queue "
                        "each); 0 = one lane per directed link on up to 8 ranks (14 at 8 ranks), world-1 "
                        "per-distance lanes beyond; a slow peer stalls only its own lane")
    p.add_argument("--host-share", action="store_true",
                   help="rccl: host-tier layers in node-shared pinned memory every rank maps; mode 0 stages one "
                        "slice per rank over its own PCIe")
    p.add_argument("--node-disk-gbps", type=float, default=0.0,
                   help="rccl: one NVMe shared by every rank of the node at this read rate (disk readers share it; "
                        "mode 3 plans it as one budget); 0 = per-rank disks")
    p.add_argument("--suspect-timeout", type=float, default=10.0,
                   help="rccl: report a P2P group stalled this long to the leader, which probes the peers and "
                        "shrinks the communicator around dead ranks (elastic recovery; 0 = only on failure)")
    p.add_argument("--inject", action="append", default=[], metavar="SPEC",
                   help="fault injection: drop-chunk=P | kill-rank=R@T | slow-link=S:D:RATE")
    p.add_argument("--job-timeout", type=float, default=0.0,
                   help="leader: re-dispatch a job not acked within this many seconds (+ bytes/--job-min-rate)")
    p.add_argument("--max-retries", type=int, default=4, help="CRC failures of one chunk before giving up")
    p.add_argument("--persist-dir", default="",
                   help="after delivery, write this node's layers + CRC manifest here; on start, announce "
                        "layers found here as disk-tier copies (resume without re-transfer)")
    p.add_argument("--seed", type=int, default=0, help="mode-1 owner RNG seed")
    p.add_argument("--owner-policy", default=None, choices=["random", "balanced", "links"],
                   help="mode 1 owner choice: random (reference), balanced (egress bytes), links (per-link time, "
                        "relays around slow links; default on the rccl engine)")
    p.add_argument("--pull-window", type=int, default=1)
    p.add_argument("--pull-job-mib", type=int, default=0,
                   help="mode 2: split layers into jobs of this many MiB (0 = one job per layer, reference)")
    p.add_argument("--bcast", default="relay", choices=["relay", "collective", "fanout"],
                   help="mode 0 on rccl: relay = scatter + peer relay over all xGMI links; collective = "
                        "ncclBroadcast per layer; fanout = leader sends every copy")
    p.add_argument("--timeout", type=float, default=3600.0)
    p.add_argument("--json-summary", action="store_true")
    return p


def engine_opts(args) -> dict:
    """Planned-engine (rccl) knobs from the CLI (bench.py shares them); the
    other PlannedConfig fields keep their defaults - set them through
    Runtime(engine_opts=...)."""
    return {"verify_cus": int(getattr(args, "verify_cus", -1)), "suspect_s": getattr(args, "suspect_timeout", 10.0),
            "lanes": int(getattr(args, "lanes", 0)), "comm_init": getattr(args, "comm_init", "split")}


def nccl_ids(core, world: int, args) -> bytes:
    """Rank 0's RCCL bootstrap ids: one per comm lane (parallel init) or one (split)."""
    n = core.resolve_lanes(world, int(getattr(args, "lanes", 0))) if getattr(args, "comm_init", "split") == "parallel" else 1
    return core.nccl_unique_id(n)


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL across rank processes
    torchrun_rank = os.environ.get("RANK")
    if args.engine == "auto":
        args.engine = "host"
        if torchrun_rank is not None:
            import torch  # device_count() does not initialise the GPU

            if torch.cuda.device_count() > 0:
                args.engine = "rccl"
    if (args.id is None and torchrun_rank is None) or (args.id is not None and args.id < 0) or not args.f:
        print(USAGE)
        print()
        return 0

    from . import _core
    from .utils.config import ConfigError, load_config

    _core.set_log_level(0 if args.v else 1)  # cmd/main.go:38-42
    try:
        cfg = load_config(args.f)
        leader = cfg.leader()
    except ConfigError as e:
        print(json.dumps({"level": "error", "error": str(e), "message": "config"}), file=sys.stderr)
        return 1
    node_ids = sorted(n.id for n in cfg.nodes)
    my_id = args.id if args.id is not None else node_ids[int(torchrun_rank)]
    try:
        me = cfg.node(my_id)
    except ConfigError as e:
        print(json.dumps({"level": "error", "error": str(e), "message": "node not found in config"}), file=sys.stderr)
        return 1

    if args.c:
        return run_client(cfg, my_id)

    from .parallel.runtime import Runtime
    from .utils.faults import arm_kill, parse_inject

    try:
        faults = parse_inject(args.inject)
    except ValueError as e:
        print(json.dumps({"level": "error", "error": str(e), "message": "--inject"}), file=sys.stderr)
        return 2

    barrier = None
    uid = None
    device = me.device
    world = int(os.environ.get("WORLD_SIZE", "1")) if torchrun_rank is not None else 1
    if args.engine == "rccl" or world > 1:
        import torch
        import torch.distributed as dist

        if args.engine == "rccl":
            from .utils.launch import rank_device

            local_rank = int(os.environ.get("LOCAL_RANK", "0"))
            device = rank_device(int(os.environ.get("RANK", "0")), local_rank, me.device)
            torch.cuda.set_device(device)
            from .utils.numa import bind_to_gpu

            bind_to_gpu(device)  # host layers on the GPU's NUMA node
        if world > 1:
            # Bootstrap only (gloo over TCP): barriers, the ncclUniqueId, addresses.
            dist.init_process_group("gloo")
            if args.engine == "rccl":
                box = [nccl_ids(_core, world, args) if dist.get_rank() == 0 else None]
                dist.broadcast_object_list(box, src=0)
                uid = box[0]
            barrier = dist.barrier
    hosts = None
    if world > 1:
        from .utils.launch import gather_hosts

        hosts = gather_hosts(my_id)  # multi-node torchrun: host-aware lanes and plans
    from .utils.launch import listen_addr as _listen_addr
    registry = cfg.registry()
    client = cfg.client(my_id)
    if client is not None:
        registry[_core.CLIENT_ID] = client.addr
    weights = None
    if args.weights:
        from .models.weights import PRESETS, layer_nbytes

        if args.weights not in PRESETS:
            print(f"error: --weights {args.weights}: presets are {', '.join(PRESETS)}", file=sys.stderr)
            return 2
        weights = PRESETS[args.weights]
        bad = {l: n for l, n in cfg.layer_sizes().items() if n != layer_nbytes(weights)}
        if bad:
            print(f"error: --weights {args.weights} needs LayerSize {layer_nbytes(weights)} "
                  f"(layers {sorted(bad)[:8]} differ)", file=sys.stderr)
            return 2
    rt = Runtime(cfg, my_id, engine=args.engine, storage_path=args.s,
                 chunk_bytes=args.chunk_mib << 20,
                 verify=args.verify != "none", registry=registry, barrier=barrier,
                 nccl_uid=uid, device=device, pack=args.pack, store=args.store,
                 inject_corrupt=faults.drop_chunk, max_retries=args.max_retries,
                 host_link_rate=faults.link_rates_from(my_id),
                 persist_dir=args.persist_dir,
                 engine_opts={**engine_opts(args), "link_rate": faults.link_rates_from(my_id)},
                 host_share=args.host_share and args.engine == "rccl", node_disk_gbps=args.node_disk_gbps,
                 node_key="c" + hashlib.blake2b((args.f + os.environ.get("MASTER_PORT", "")).encode(),
                                                digest_size=6).hexdigest(),
                 layer_source=_weights_source(weights) if weights is not None else None, hosts=hosts,
                 listen_addr=None if me.addr or not hosts else _listen_addr(True))
    if barrier is not None:
        # torchrun: nodes without a fixed Addr listen on ephemeral ports; share them.
        import torch.distributed as dist

        pairs = [None] * dist.get_world_size()
        from .utils.launch import advertised

        dist.all_gather_object(pairs, (my_id, advertised(rt.transport.address())))
        reg = dict(registry)
        reg.update({nid: addr for nid, addr in pairs})
        rt.transport.set_registry(reg)
        if args.host_share:
            barrier()  # every rank mapped the shared host layers: drop their names
            rt.unlink_shared()
    if args.l:
        print(json.dumps({"level": "info", "node": my_id, "message": "layer set up"}), file=sys.stderr)
        rt.close()
        return 0
    role = "leader" if my_id == leader.id else "receiver"
    print(f"launching {role}...\n[addr: {rt.transport.address()}, id: {my_id}, filename: {args.f}, "
          f"storagePath: {args.s}, mode: {args.m}]", flush=True)
    if args.m not in (0, 1, 2, 3):
        print(json.dumps({"level": "error", "node": my_id, "error": "unknown mode", "message": f"{role} failed"}),
              file=sys.stderr)
        return 1
    if args.owner_policy is None:
        args.owner_policy = "links" if args.engine == "rccl" else "random"
    policy = dict(seed=args.seed, owner_policy=args.owner_policy, pull_window=args.pull_window,
                  relay=args.bcast != "fanout", collective=args.bcast == "collective",
                  job_timeout_s=args.job_timeout, pull_job_bytes=args.pull_job_mib << 20)
    rt.prepare(args.m, **policy)
    if barrier:
        barrier()
    # The kill clock starts once this node is sending layer bytes (not at process start).
    arm_kill(faults, my_id, started=lambda: rt.transport.bytes_sent > (64 << 10)
             or (rt.engine is not None and rt.engine.stats().bytes_sent > 0))
    res = rt.execute(args.timeout, announce_retry_s=30.0)
    if role == "leader" and res.ok:
        print(f"Time to deliver: {go_duration(res.time_to_deliver_s)}", flush=True)
        if args.json_summary:
            gbps = res.bytes_planned / res.time_to_deliver_s / 1e9 if res.time_to_deliver_s > 0 else 0.0
            summary = {"time_to_full_placement_s": res.time_to_deliver_s, "aggregate_GBps": gbps,
                       "bytes_moved": res.bytes_planned, "ranks": len(cfg.nodes), "mode": args.m,
                       "engine": args.engine, "pack": args.pack, "plan_ms": res.plan_ms,
                       "nacks": res.nacks, "redispatched": res.redispatched, "recoveries": res.recoveries,
                       "dropped": res.dropped}
            if res.engine_stats:
                summary["engine"] = {"name": args.engine, **res.engine_stats}
            print(json.dumps(summary), flush=True)
    if not res.ok:
        print(json.dumps({"level": "error", "node": my_id, "error": res.error, "message": f"{role} failed"}),
              file=sys.stderr)
    elif weights is not None and cfg.assignment.get(my_id):
        _check_weights(rt, weights, cfg.assignment[my_id], my_id)
    if args.persist_dir and cfg.assignment.get(my_id) and (res.ok or rt.engine is not None):
        # After a failed session the planned engines keep what did land, chunk
        # by chunk: the next run with the same --persist-dir resumes from there.
        try:
            done = rt.persist(partial=not res.ok)
            print(json.dumps({"level": "info", "node": my_id, "layers": done, "dir": args.persist_dir,
                              "partial": not res.ok, "message": "layers persisted"}), file=sys.stderr)
        except Exception as e:  # noqa: BLE001 - a failed session must still exit cleanly
            print(json.dumps({"level": "error", "node": my_id, "error": str(e)[:300],
                              "message": "persist failed"}), file=sys.stderr)
    if barrier:
        # A rank may have died during the session (elastic recovery): do not
        # wait for it forever.
        try:
            import torch.distributed as dist

            dist.monitored_barrier(timeout=datetime.timedelta(seconds=15))
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"level": "warn", "node": my_id, "error": str(e)[:200],
                              "message": "final barrier incomplete (a rank is gone)"}), file=sys.stderr)
    time.sleep(0.05)  # let startup messages flush before sockets close
    rt.close()
    return 0 if res.ok else 1


def _weights_source(spec):
    """layer_source for --weights: layer l = random-init weights seeded by l."""
    from .models.weights import flatten, random_layer

    return lambda l, n: flatten(random_layer(spec, 1000 + l), spec)


def _check_weights(rt, spec, layers, my_id: int) -> None:
    """Serving smoke: each assigned layer as named parameters (zero-copy views in
    HBM on the rccl engine), one forward pass, compared with the same pass on the
    seeded weights."""
    import torch

    from .models.weights import decoder_forward, random_layer

    x = torch.randn(1, 8, spec.hidden, generator=torch.Generator().manual_seed(0)).to(torch.bfloat16)
    worst = 0.0
    for l in sorted(layers):
        p = rt.layer_params(l, spec)
        dev = next(iter(p.values())).device
        y = decoder_forward(x.to(dev), p, spec).float().cpu()
        y0 = decoder_forward(x, random_layer(spec, 1000 + l), spec).float()
        worst = max(worst, float((y - y0).norm() / y0.norm()))
    print(json.dumps({"level": "info", "node": my_id, "layers": len(layers), "preset": spec.name,
                      "max_rel_err": worst, "message": "weights forward check"}), file=sys.stderr, flush=True)


def run_client(cfg, node_id: int) -> int:
    """cmd/main.go:69-91: external client serving rate-limited in-memory layers to its node."""
    from . import _core
    from .parallel.runtime import layer_seed

    cc = cfg.client(node_id)
    if cc is None:
        print(json.dumps({"level": "info", "message": "external client not found in config"}), file=sys.stderr)
        return 1
    node = cfg.node(node_id)
    t = _core.tcp_transport(cc.addr or "127.0.0.1:0", {node_id: node.addr}, True)
    layers = {
        l: _core.LayerSrc.inmem(_core.fill_random_host(cfg.layer_size, layer_seed(0, l)), rate)
        for l, rate in cc.layers.items()
    }
    client = _core.ClientNode(node_id, t, layers)
    client.start()
    stop = {"flag": False}
    signal.signal(signal.SIGTERM, lambda *_: stop.update(flag=True))
    try:
        while not stop["flag"]:
            time.sleep(0.2)  # select {} (serve forever)
    except KeyboardInterrupt:
        pass
    client.stop()
    t.close()
    return 0


def entry() -> None:
    """Console script `dissem` (pyproject.toml)."""
    sys.exit(main())


if __name__ == "__main__":
    sys.exit(main())
