#!/usr/bin/env python3
"""Headline benchmark: aggregate GB/s + time-to-full-placement of 80 x 1 GiB
layers, mode 1 (peer retransmission), one rank per MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` runs N
ranks of one node (torchrun for N > 1). A *step* is one complete dissemination
session: every rank announces, the leader plans mode-1 retransmissions, layers
move into every GPU's HBM (host->HBM staging over PCIe, GPU->GPU over RCCL/xGMI),
every chunk is CRC32C-verified on the receiving GPU, all ranks ack, and the
leader broadcasts startup. W untimed warmup steps, then K steps, each bracketed
by barrier + device synchronize on both sides; the slowest rank's time counts.

Workload (BASELINE.json config #3, weak scaling): 80 layers x 1 GiB of random
bytes; InitialLayers seeded by a balanced random permutation into the pinned
host memory of the ranks (each rank holds 80/N layers); the Assignment gives
every rank all 80 layers (full replication, DP-serving placement). Each GPU
therefore receives 80 GiB into HBM per step at every N: at N = 1 all of it
crosses PCIe; at N = 8, 10 GiB per GPU crosses PCIe and 70 GiB arrives over
xGMI. value = N x 80 GiB / step time (GB/s, 1e9 bytes).
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
BASELINE_METRIC = "aggregate GB/s + time-to-full-placement, 80×1 GiB layers, mode 1, 8 ranks"
PROBE_BYTES = 4 << 30  # node NVMe probe file (N > 1, --tier disk): past typical drive caches


def metric_name(layers: int, layer_mib: int, mode: int, ranks: int) -> str:
    """BASELINE.json's metric with the workload and rank count this run measured
    (equal to BASELINE_METRIC for the headline config at 8 ranks)."""
    size = f"{layer_mib // 1024} GiB" if layer_mib % 1024 == 0 else f"{layer_mib} MiB"
    return (f"aggregate GB/s + time-to-full-placement, {layers}×{size} layers, mode {mode}, "
            f"{ranks} rank{'s' if ranks != 1 else ''}")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE or 1)")
    p.add_argument("--steps", type=int, default=5, help="timed sessions")
    p.add_argument("--warmup", type=int, default=1, help="untimed sessions first")
    p.add_argument("--mode", type=int, default=1, choices=[0, 1, 2, 3],
                   help="distribution mode (BASELINE config #3: 1, peer retransmission)")
    p.add_argument("--layers", type=int, default=80, help="layers (config #3: 80)")
    p.add_argument("--layer-mib", type=int, default=1024, help="MiB per layer (config #3: 1 GiB)")
    p.add_argument("--chunk-mib", type=int, default=64,
                   help="chunk grid: P2P message, CRC unit and staging copy. N = 1 reads the same at 32-256 "
                        "(56.87-56.98 GB/s, profiles/r5_chunk/). REAL-NODE GUESS at N > 1: settled by "
                        "config.per_link_busy_GBps")
    p.add_argument("--tier", default="host", choices=["host", "device", "disk"],
                   help="where the seeded layers live: pinned host memory (config #3), HBM, NVMe (config #4)")
    p.add_argument("--seeding", default="random", choices=["random", "leader", "uniform"],
                   help="InitialLayers: balanced random permutation (config #3), all on the leader (config #2), "
                        "or i.i.d. uniform owners")
    p.add_argument("--copies", type=int, default=1, help="holders per layer in the initial seeding")
    p.add_argument("--owner-policy", default="links", choices=["random", "balanced", "links"],
                   help="mode 1 owner choice when a layer has several holders (--copies > 1); links also "
                        "relays around links the plan knows to be slow")
    p.add_argument("--timeout", type=float, default=120.0,
                   help="seconds one session (step) may take before the rank gives up (also the P2P group timeout)")
    p.add_argument("--pull-window", type=int, default=0,
                   help="mode 2 jobs in flight per sender (0 = two per peer). Round-5 sim (closed loop on, 50 GB/s "
                        "links): N = 8: 7 -> 262-270 ms, 10 -> 248, 14 -> 245, 21 -> 270; N = 4: 3 -> 589, 6 -> 465; "
                        "N = 2: 1 -> 1794, 2 -> 875 (a rank's loads of its own layers hold window slots too; "
                        "profiles/r5_predict_mode2_windows.jsonl). REAL-NODE GUESS: settled by "
                        "config.per_link_busy_GBps in mode 2")
    p.add_argument("--storage", default="", help="disk tier directory")
    p.add_argument("--allow-buffered", action="store_true",
                   help="--tier disk: accept a run whose layer files sit on a memory file system or were read "
                        "without O_DIRECT (the JSON says so); by default such a run fails, since its rate is not a disk's")
    p.add_argument("--bcast", default="relay", choices=["relay", "collective", "fanout"],
                   help="mode 0: scatter+relay P2P, ncclBroadcast, or leader fan-out")
    p.add_argument("--pack", default="none", choices=["none", "fp8"],
                   help="fp8: layers are bf16 sources packed to block-scaled e4m3fn while staging "
                        "(HBM + wire format; BASELINE config #5)")
    p.add_argument("--store", default="packed", choices=["packed", "bf16"],
                   help="with --pack fp8: bf16 = every resident chunk is also dequantized to bf16 in HBM by the "
                        "fused verify+unpack kernel (the receive path of an inference deployment)")
    p.add_argument("--host-share", action="store_true",
                   help="host-tier layers in node-shared pinned memory (POSIX shm, hipHostRegister in every rank); "
                        "mode 0 then stages one slice of every layer per rank over its own PCIe (config #2)")
    p.add_argument("--node-disk-gbps", type=float, default=None,
                   help="--tier disk: the node's one NVMe read rate (GB/s) shared by every rank's disk readers and "
                        "planned as one budget by mode 3 (0 = per-rank, unpaced). Default: unpaced at N = 1 (one rank "
                        "has the NVMe alone; paced at 13.3 it read exactly 13.30 GB/s, unpaced 20.3, "
                        "profiles/r5_disk/); at N > 1 MEASURED before the run by an O_DIRECT read probe on each host "
                        "(utils/diskprobe.py; JSON node_disk_GBps, node_disk_source)")
    # Defaults measured on a real MI355X cite their evidence; the ones only a
    # real 8-GPU node can settle name the JSON field that will (REAL-NODE GUESS).
    p.add_argument("--verify-cus", type=int, default=-1,
                   help="the verify stream runs on the last N CUs only, RCCL lanes and copies on the others (-1: 32, "
                        "4 CUs on each XCD, when N > 1 - 128 with --store bf16 - and 0 alone; 0: all shared). "
                        "Evidence: bin/contention on one MI355X, a 64-workgroup copy keeps 99.6 %% of its rate "
                        "beside 450 GB/s of verify on the last 32 CUs (profiles/r4_contention); the fused bf16 "
                        "verify needs 128 at 7 x 153 GB/s of ingress (scripts/verify_bench.py --cus 128). "
                        "REAL-NODE GUESS at N = 8: settled by config.verify_busy_frac_rank0 and per_link_busy_GBps")
    p.add_argument("--lanes", type=int, default=0,
                   help="comm lanes (RCCL communicator + stream + dedicated HW queue each); 0 = one lane per "
                        "directed link on up to 8 ranks (14 at N = 8), world-1 per-distance lanes beyond. "
                        "REAL-NODE GUESS (schedule evidence: the sim's RCCL round model, tests/test_timing_sim.py); "
                        "settled by config.per_link_busy_GBps and comm_init_ms_per_lane / comm_connect_ms_per_lane")
    p.add_argument("--probe-mib", type=int, default=256,
                   help="N > 1: untimed pre-flight probe of every directed link with this many MiB "
                        "(all lanes at once, then each pair alone); 0 = skip. Its rates floor the closed loop's "
                        "link capacities for the first sessions. REAL-NODE GUESS for the size: settled by "
                        "config.probe_lane_GBps (concurrent vs solo) against per_link_busy_GBps")
    p.add_argument("--inject", action="append", default=[], metavar="SPEC",
                   help="fault injection (utils/faults.py), e.g. slow-link=0:1:20G (rank 0 -> 1 capped at 20 GB/s)")
    p.add_argument("--source-pool", type=int, default=0,
                   help="host tier: layers share this many distinct pinned source buffers (layer l holds "
                        "pool buffer l %% P: random bytes, identical across layers of one residue) - fits "
                        "126 x 3 GiB bf16 sources in host memory; 0 = one buffer per layer. Keep P at least the "
                        "largest pool that fits: 8-20 layer runs lose 9-17%% of PCIe throughput when layers "
                        "share buffers (profiles/r2_pool_share20; the 126-layer preset does not)")
    p.add_argument("--preset", default="", choices=["", "llama70b", "llama405b-fp8"],
                   help="llama70b = 80 x 1 GiB (default); llama405b-fp8 = 126 x 3 GiB with --pack fp8")
    args = p.parse_args(argv)
    if args.preset == "llama405b-fp8":
        args.layers, args.layer_mib, args.pack = 126, 3072, "fp8"
    elif args.preset == "llama70b":
        args.layers, args.layer_mib = 80, 1024
    return args


def relaunch_with_torchrun(args) -> int:
    # Launched for N > 1 without torchrun: start it as a child (never exec after GPU init).
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def load_supervise():
    """utils/supervise.py on its own: a supervisor imports neither the package
    (its __init__ loads the native runtime) nor anything that touches the GPU."""
    import importlib.util

    name = "dld_supervise"
    if name not in sys.modules:
        spec = importlib.util.spec_from_file_location(
            name, os.path.join(HERE, "distributed_llm_dissemination_amd", "utils", "supervise.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
    return sys.modules[name]


def fallback_attempts(args, world):
    """The supervised attempts at N > 1: as asked; then round 2's data plane
    (one lane per ring distance - world-1 communicators and HW queues instead
    of 14); then that without RCCL's P2P/IPC transport (host shared memory
    between the GPUs). Lane communicators are split from the world one."""
    Attempt = load_supervise().Attempt
    atts = [Attempt("")]
    if args.lanes == 0 and world > 2:
        atts.append(Attempt(f"lanes={world - 1}", ["--lanes", str(world - 1)]))
    atts.append(Attempt(f"lanes={world - 1}, NCCL_P2P_DISABLE=1", ["--lanes", str(world - 1)],
                        {"NCCL_P2P_DISABLE": "1"}))
    return atts


def supervise(args, world, rank) -> int:
    """torchrun rank process at N > 1: never touches the GPU; runs this rank's
    worker in fresh child processes until an attempt succeeds (utils/supervise.py)."""
    import tempfile

    sup = load_supervise()

    def log(msg):
        print(f"[bench supervisor {rank}] {msg}", file=sys.stderr, flush=True)

    json_path = os.path.join(tempfile.gettempdir(), f"dld_bench_{os.getpid()}.json") if rank == 0 else None
    rc, hist = sup.run_attempts([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                            fallback_attempts(args, world), json_path=json_path, log=log)
    if rank == 0:
        if rc == 0 and not sup.emit_json(json_path):
            log("the successful attempt left no result line")
            rc = 1
        if json_path and os.path.exists(json_path):
            os.unlink(json_path)
    return rc


def main(argv=None) -> int:
    args = parse_args(argv)
    # RCCL's cross-process buffer sharing on these hosts needs dmabuf IPC (the
    # legacy IPC path fails in hipIpcGetMemHandle: tests/test_gpu_ipc.py,
    # profiles/r3_ipc/); set before any HIP init and inherited by every child.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is None:
        args.gpus = world
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch_with_torchrun(args)
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    sys.path.insert(0, HERE)
    sup = load_supervise()

    if world > 1 and not os.environ.get(sup.ENV_PREFIX) and sup.agent_store_available():
        return supervise(args, world, rank)
    chan = sup.WorkerChannel.from_env()
    try:
        return worker(args, world, rank, chan)
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 - report any failure to the supervisors, then exit non-zero
        import traceback

        traceback.print_exc()
        if chan is not None:
            chan.fail(f"{type(e).__name__}: {e}")
            sys.stderr.flush()
            os._exit(1)  # a stalled lane's kernels would hang the runtime's teardown
        raise


def worker(args, world, rank, chan) -> int:
    # stdout carries exactly one JSON line (rank 0): everything else any library
    # prints there (RCCL's version banner, gloo) goes to stderr.
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    from distributed_llm_dissemination_amd.utils.launch import advertised, gather_hosts, listen_addr, rank_device, shared_gpu

    beat = chan.heartbeat if chan is not None else (lambda phase: None)
    beat("start")
    local_rank = rank_device(rank, int(os.environ.get("LOCAL_RANK", str(rank))))
    import torch
    import torch.distributed as dist

    from distributed_llm_dissemination_amd import _core
    from distributed_llm_dissemination_amd.models.catalog import delivered_bytes, make_workload
    from distributed_llm_dissemination_amd.__main__ import engine_opts
    from distributed_llm_dissemination_amd.parallel.runtime import Runtime
    from distributed_llm_dissemination_amd.utils.faults import parse_inject

    faults = parse_inject(args.inject)

    _core.set_log_level(int(os.environ.get("DISSEM_LOG_LEVEL", "2")))  # 1 = info, 0 = debug

    def log(msg):
        print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True)

    def failed(why):
        log(why)
        if chan is not None:
            chan.fail(why)
            sys.stderr.flush()
            os._exit(1)
        raise SystemExit(1)

    if not torch.cuda.is_available():
        print("error: no GPU visible", file=sys.stderr)
        return 2
    torch.cuda.set_device(local_rank)
    # pinned host layers on the GPU's NUMA node (allocated below, on this thread)
    from distributed_llm_dissemination_amd.utils.numa import bind_to_gpu

    numa = bind_to_gpu(local_rank)
    if world > 1:
        if chan is not None:
            dist.init_process_group("gloo", store=chan.pg_store(), rank=rank, world_size=world)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        barrier = dist.barrier
    else:
        barrier = lambda: None  # noqa: E731
    # ranks on several machines (multi-node torchrun): host-aware lanes and plans
    hosts = gather_hosts(rank) if world > 1 else None
    beat("setup")
    if chan is not None and chan.attempt in faults.fail_attempts.get(rank, []):
        failed(f"fault injection: fail-attempt={rank}@{chan.attempt}")

    layer_bytes = args.layer_mib << 20
    cfg = make_workload(world, args.layers, layer_bytes, seeding=args.seeding, tier=args.tier, copies=args.copies,
                        seed=0, assignment="replicate", chunk_bytes=args.chunk_mib << 20)
    total_bytes = delivered_bytes(cfg)

    from distributed_llm_dissemination_amd.__main__ import nccl_ids

    uid = nccl_ids(_core, world, args) if (world > 1 and rank == 0) else None
    if world > 1:
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    free, tot = _core.mem_info()
    log(f"HBM free {free / 2**30:.1f} / {tot / 2**30:.1f} GiB; setting up {args.layers} x {args.layer_mib} MiB"
        + (f" (attempt {chan.attempt}: {chan.label})" if chan is not None and chan.label else ""))
    t_setup = time.time()
    # names the node-shared resources of this run (shm segments, disk pacer): same on every rank
    import hashlib

    run_tag = os.environ.get("DLD_SUP_PREFIX", "") + os.environ.get("MASTER_PORT", "") + os.environ.get(
        "TORCHELASTIC_RUN_ID", "") if world > 1 else str(os.getpid())
    node_key = "b" + hashlib.blake2b(run_tag.encode(), digest_size=6).hexdigest()
    disk_info = {}  # --tier disk: storage, read mode and page-cache facts for the JSON
    disk_gbps = args.node_disk_gbps if args.node_disk_gbps is not None else 0.0
    disk_source = "flag" if args.node_disk_gbps is not None else "unpaced"
    if args.tier == "disk" and args.node_disk_gbps is None and world > 1:
        # the node's one NVMe, shared by every rank: measured once per host
        # (utils/diskprobe.py), the slowest host's rate for all; 13.3 (the
        # round-1 box, profiles/r1_diskspeed.log) where O_DIRECT is unavailable
        from distributed_llm_dissemination_amd.utils.diskprobe import read_rate_gbps

        mine = None
        if int(os.environ.get("LOCAL_RANK", "0")) == 0:  # one probe per host (ranks sharing a GPU included)
            try:  # never leave the other ranks waiting in the gather below
                mine = read_rate_gbps(args.storage or os.path.join(os.getcwd(), "storage"), size_bytes=PROBE_BYTES)
            except Exception as e:  # noqa: BLE001 - e.g. a full or read-only disk: keep the default
                log(f"node NVMe probe failed: {e}")
            log(f"node NVMe read rate: {mine if mine is None else round(mine, 2)} GB/s (O_DIRECT probe)")
        rates = [None] * world
        dist.all_gather_object(rates, mine)
        got = [r for r in rates if r]
        disk_gbps, disk_source = (min(got), "measured") if got else (13.3, "default")
        if got:
            disk_info["node_disk_probe_GiB"] = PROBE_BYTES / 2**30  # the probe file's size beside its rate
    if args.tier == "disk":
        from distributed_llm_dissemination_amd.utils.config import SOURCE_DISK
        from distributed_llm_dissemination_amd.utils.diskprobe import refusal, storage_info

        st = storage_info(args.storage or os.path.join(os.getcwd(), "storage"))
        mine_bytes = sum(cfg.node(rank).initial_layers.get(SOURCE_DISK, {}).values())
        fit = int(st["avail_bytes"] * 0.97 // layer_bytes)
        disk_info.update({"storage_fs": st["fs"], "storage_device": st["device"], "storage_mount": st["mount"],
                          "storage_avail_GB": round(st["avail_bytes"] / 1e9, 1), "layers_fit_on_storage": fit,
                          **({"storage_note": st["note"]} if "note" in st else {})})
        log(f"disk tier on {st['mount']} ({st['fs']}, {st['device']}): {st['avail_bytes'] / 1e9:.1f} GB free, "
            f"this rank writes {mine_bytes / 1e9:.1f} GB")
        why = refusal(st["fs"], "o_direct", args.allow_buffered)
        if why:
            failed(f"--tier disk: {why}; pass --allow-buffered to run anyway")
        if mine_bytes > st["avail_bytes"] * 0.97:
            failed(f"--tier disk: this rank's {mine_bytes / 1e9:.1f} GB of layer files do not fit the "
                   f"{st['avail_bytes'] / 1e9:.1f} GB free on {st['mount']} (at most {fit} layers of "
                   f"{args.layer_mib} MiB): pass --layers {fit} or another --storage")
    rt = Runtime(cfg, rank, engine="rccl", transport="tcp", chunk_bytes=args.chunk_mib << 20,
                 verify=True, payload_seed=0, registry={rank: listen_addr(bool(hosts))},
                 barrier=barrier, nccl_uid=uid, device=local_rank, storage_path=args.storage, pack=args.pack,
                 store=args.store, group_timeout_s=min(300.0, args.timeout),
                 engine_opts={**engine_opts(args), "link_rate": faults.link_rates_from(rank)},
                 inject_corrupt=faults.drop_chunk, source_pool=args.source_pool, host_share=args.host_share,
                 node_key=node_key, node_disk_gbps=disk_gbps, hosts=hosts)
    beat("comm ready")
    if args.pack != "none":
        # bytes that land in HBM (and cross PCIe/xGMI) are the packed ones
        src_bytes = total_bytes
        total_bytes = src_bytes * rt.slot_sizes[0] // rt.sizes[0]
    if world > 1:
        addrs = [None] * world
        dist.all_gather_object(addrs, advertised(rt.transport.address()))
        rt.transport.set_registry({i: a for i, a in enumerate(addrs)})
    if args.host_share:
        barrier()  # every rank has mapped the shared segments: drop their names
        rt.unlink_shared()
    log(f"setup done in {time.time() - t_setup:.1f}s")

    probe = {}
    if world > 1 and args.probe_mib > 0:
        beat("probe")
        try:
            probe = rt.probe_links(args.probe_mib << 20, timeout_s=30.0)
        except RuntimeError as e:
            failed(str(e))
        log(f"link probe: {probe.get('probe_ms')} ms; concurrent GB/s {probe.get('concurrent')}")
        # the probe's concurrent rates floor the closed-loop link capacities (B/s)
        rt.observe_probe({p: g * 1e9 for p, g in probe.get("concurrent", {}).items() if g},
                         {p: g * 1e9 for p, g in probe.get("concurrent_in", {}).items() if g})

    engine_note = f"{rt.engine.stats().lanes} comm lanes" if world > 1 else ""
    policy = dict(seed=0, pull_window=args.pull_window or max(1, 2 * (world - 1)),
                  owner_policy=args.owner_policy,
                  relay=args.bcast == "relay", collective=args.bcast == "collective",
                  adapt_links=True, hierarchical=True)

    cache_left = []  # --tier disk: fraction of a layer file still in the page cache before each session

    def step(timed: bool, i: int):
        beat(f"{'step' if timed else 'warmup'} {i}")
        if args.tier == "disk":
            cache_left.append(rt.drop_disk_cache())  # conf/exe.sh:17: every run starts cold
        rt.prepare(args.mode, **policy)
        barrier()
        torch.cuda.synchronize()
        _core.trace_push("bench.step" if timed else "bench.warmup")
        t0 = time.perf_counter()
        res = rt.execute(args.timeout)
        torch.cuda.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        _core.trace_pop()
        if not res.ok:
            failed(f"session failed on rank {rank}: {res.error}")
        return dt, res

    for i in range(args.warmup):
        dt, res = step(False, i)
        log(f"warmup {i}: {dt * 1e3:.1f} ms ({total_bytes / dt / 1e9:.1f} GB/s)")
    links0 = rt.link_stats()
    times = []
    plans = []  # leader (rank 0): the plan of every timed step - it runs after "timer start"
    last = None
    disk_bytes = {"direct": 0, "buffered": 0}
    for i in range(args.steps):
        dt, last = step(True, i)
        times.append(dt)
        plans.append(last)
        disk_bytes["direct"] += last.engine_stats.get("disk_direct_bytes", 0)
        disk_bytes["buffered"] += last.engine_stats.get("disk_buffered_bytes", 0)
        log(f"step {i}: {dt * 1e3:.1f} ms ({total_bytes / dt / 1e9:.1f} GB/s) ttd={last.time_to_deliver_s * 1e3:.1f} ms")
    beat("measured")
    if args.tier == "disk":
        if world > 1:
            got = [None] * world
            dist.all_gather_object(got, (disk_bytes, max(cache_left, default=-1.0)))
            disk_bytes = {k: sum(g[0][k] for g in got) for k in disk_bytes}
            left = max(g[1] for g in got)
        else:
            left = max(cache_left, default=-1.0)
        from distributed_llm_dissemination_amd.utils.diskprobe import read_mode, refusal

        mode_ = read_mode(disk_bytes["direct"], disk_bytes["buffered"])
        disk_info.update({"disk_read_mode": mode_, "disk_direct_GB": round(disk_bytes["direct"] / 1e9, 2),
                          "disk_buffered_GB": round(disk_bytes["buffered"] / 1e9, 2),
                          "page_cache_dropped": left >= 0, "page_cache_resident_max": round(left, 4)})
        why = refusal(disk_info["storage_fs"], mode_, args.allow_buffered)
        if why:
            failed(f"--tier disk: {why} ({disk_bytes['buffered'] / 1e9:.1f} GB buffered); pass --allow-buffered "
                   f"to report it anyway")
    total = sum(times)
    # Per directed link over the timed steps: bytes this rank sent to each peer,
    # and the device time of the P2P groups that sent to it.
    links1 = rt.link_stats()
    mine = {p: (links1["sent"].get(p, 0) - links0["sent"].get(p, 0),
                links1["send_busy_ms"].get(p, 0.0) - links0["send_busy_ms"].get(p, 0.0)) for p in links1["sent"]}
    all_links = [mine]
    all_probe = [probe]
    init_ms = [rt.engine.stats().comm_init_ms]
    if world > 1:
        t = torch.tensor([total], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        total = float(t.item())
        all_links = [None] * world
        dist.all_gather_object(all_links, mine)
        all_probe = [None] * world
        dist.all_gather_object(all_probe, probe)
        init_ms = [None] * world
        dist.all_gather_object(init_ms, rt.engine.stats().comm_init_ms)
    ms_per_step = total / max(1, args.steps) * 1e3
    value = total_bytes * args.steps / total / 1e9
    if rank == 0:
        out = {
            "metric": metric_name(args.layers, args.layer_mib, args.mode, world),
            "baseline_metric": BASELINE_METRIC,  # BASELINE.json's name; `metric` says what this run measured
            "ranks": world,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic: random-byte layers (splitmix64), balanced random seeding in pinned host memory",
            "config": {
                "model": f"{args.layers}x{args.layer_mib}MiB layers (Llama-3-70B-sized shards)",
                "global_batch": None,
                "seq_len": None,
                "parallelism": f"dp{world} (full replication)",
                "mode": args.mode,
                "tier": args.tier,
                "seeding": args.seeding,
                "chunk_mib": args.chunk_mib,
                "verify": True,
                "bytes_per_step": total_bytes,
                "time_to_full_placement_s": round(ms_per_step / 1e3, 6),
                "leader_time_to_deliver_s": round(last.time_to_deliver_s, 6) if last else None,
                "engine": ("rccl-socket, all ranks on one GPU (schedule rehearsal; bandwidth not meaningful)"
                           if world > 1 and shared_gpu() else
                           "rccl-p2p-xgmi" if world > 1 else "hip-h2d (no peers)") + (
                               f", {engine_note}" if engine_note else ""),
                "pack": args.pack,
                "payload": "bf16 layer shards as raw bytes, moved bit-exact (CRC32C per chunk)",
                **({"host_share": True} if args.host_share else {}),
                **({"node_disk_GBps": round(disk_gbps, 2), "node_disk_source": disk_source, **disk_info}
                   if args.tier == "disk" else {}),
            },
        }
        if args.pack != "none":
            out["dtype"] = "fp8"
            out["config"]["payload"] = "bf16 sources packed on the GPU to fp8 e4m3fn, one power-of-two scale per block"
            out["config"]["model"] = f"{args.layers}x{args.layer_mib}MiB bf16 layers (Llama-3.1-405B-sized shards), fp8 in HBM"
            out["config"]["bf16_source_bytes_per_step"] = src_bytes
            out["config"]["bf16_equivalent_GBps"] = round(src_bytes * args.steps / total / 1e9, 3)
            out["config"]["store"] = args.store
        if last is not None and last.engine_stats:
            out["config"]["engine_stats_rank0"] = last.engine_stats
            vb = last.engine_stats.get("verify_busy_ms")
            if vb is not None and last.seconds > 0:  # occupancy of the verify CUs in the last session
                out["config"]["verify_busy_frac_rank0"] = round(vb / (last.seconds * 1e3), 3)
            nck = last.engine_stats.get("verify_chunks")
            if vb is not None and nck:  # device time of the batched checks per checked chunk
                out["config"]["verify_us_per_chunk_rank0"] = round(vb * 1e3 / nck, 1)
                calls = last.engine_stats.get("verify_calls") or 0
                if calls:  # the batching behind that rate: chunks per verify launch
                    out["config"]["verify_chunks_per_call_rank0"] = round(nck / calls, 2)
            st = last.engine_stats.get("bytes_staged")
            if st and last.seconds > 0:  # this rank's host -> HBM rate over the session (PCIe bound: ~57 GB/s)
                out["config"]["stage_GBps_rank0"] = round(st / last.seconds / 1e9, 2)
        if plans:
            # the leader's plan inside the timed window (reference: node.go:1161-1165 starts the
            # timer before the solve, :1225-1231 logs its computation time)
            pm = [p.plan_ms for p in plans]
            out["config"]["plan"] = {
                "ms_mean": round(sum(pm) / len(pm), 3), "ms_max": round(max(pm), 3),
                "sched_ms_mean": round(sum(p.plan_sched_ms for p in plans) / len(plans), 3),
                "dispatch_ms_mean": round(sum(p.plan_dispatch_ms for p in plans) / len(plans), 3),
                "cached_steps": sum(1 for p in plans if p.plan_cached),
                "solver": plans[-1].plan_solver,
            }
        out["config"]["numa_rank0"] = numa  # {} when the GPU's node is unknown or outside this cpuset
        if chan is not None:
            out["config"]["fallback"] = chan.label or None
            out["config"]["failed_attempts"] = chan.history
        if world > 1:
            es = rt.engine.stats()
            out["config"]["comm_lanes"] = es.lanes
            out["config"]["comm_init_ms_rank0"] = round(es.comm_init_ms, 1)
            out["config"]["comm_init_ms_max"] = round(max(init_ms), 1)
            out["config"]["comm_connect_ms_rank0"] = round(es.comm_connect_ms, 1)
            # per lane, rank 0: communicator set-up and connects (settles parallel vs split on a real node)
            out["config"]["comm_init_ms_per_lane"] = [round(x, 1) for x in es.lane_init_ms]
            out["config"]["comm_connect_ms_per_lane"] = [round(x, 1) for x in es.lane_connect_ms]
            out["config"]["comm_init"] = "split"
            # the verify stream's CUs (the last ones of the mask; RCCL and copies on the rest)
            out["config"]["verify_cus"] = (args.verify_cus if args.verify_cus >= 0
                                           else 128 if args.store == "bf16" else 32)
            if hosts:
                out["config"]["hosts"] = len(set(hosts.values()))
        if world > 1:
            # GB/s per directed link: averaged over the timed wall time, and while
            # its send groups were on the device (busy).
            wall, busy = {}, {}
            for src, per in enumerate(all_links):
                for p, (b, ms) in sorted(per.items()):
                    wall[f"{src}->{p}"] = round(b / total / 1e9, 2)
                    busy[f"{src}->{p}"] = round(b / (ms / 1e3) / 1e9, 2) if ms > 0 else None
            out["config"]["per_link_GBps"] = wall
            out["config"]["per_link_busy_GBps"] = busy
            # the per directed link rates the leader's last plan used (measured, closed loop)
            plan = rt.plan_link_bw()
            out["config"]["adapt_links"] = True
            out["config"]["plan_link_GBps"] = {f"{a}->{b}": round(v / 1e9, 2) for (a, b), v in sorted(plan.items())}
            if any(all_probe):
                # untimed pre-flight probe: GB/s per directed link (sender's device time)
                pr = {"MiB": args.probe_mib, "concurrent": {}, "solo": {}}
                for src, p in enumerate(all_probe):
                    for kind in ("concurrent", "solo"):
                        for dst, gbps in sorted((p or {}).get(kind, {}).items()):
                            pr[kind][f"{src}->{dst}"] = gbps
                pr["probe_ms_max"] = max((p or {}).get("probe_ms", 0) for p in all_probe)
                out["config"]["probe_lane_GBps"] = pr
        line = json.dumps(out) + "\n"
        json_file = os.environ.get("DLD_SUP_JSON")
        if chan is not None and json_file:
            with open(json_file + ".tmp", "w") as f:
                f.write(line)
            os.replace(json_file + ".tmp", json_file)
            chan.ok()
        else:
            json_out.write(line)
            json_out.flush()
    beat("teardown")
    rt.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
