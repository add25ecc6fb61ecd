"""Per-rank runtime: materialize layers, build the transport + data engine, and
run dissemination sessions (reference: cmd/main.go:23-220).

One process per node (per GPU on MI355X). The control plane is the C++ TCP
transport (JSON envelopes, reference wire format). The data plane is either

* ``host``: the C++ host engine (layer bytes over TCP, host RAM target) - the
  reference's behavior, used for CPU runs (BASELINE config #1) and tests; or
* ``rccl``: the C++ GPU engine (RCCL P2P over xGMI into HBM, pinned-host/NVMe
  staging, CRC32C verify kernel), the MI355X data plane.

A *session* is one full dissemination: announce -> schedule -> transfer ->
ack -> startup, with "Time to deliver" measured by the leader. Transports and
the GPU engine persist across sessions; each session gets a fresh Node and a
new epoch so stray messages from an earlier session are dropped.
"""

from __future__ import annotations

import hashlib
import json
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from .. import _core
from ..utils.config import (
    SOURCE_CLIENT,
    SOURCE_DEVICE,
    SOURCE_DISK,
    Config,
)

MiB = 1 << 20


def layer_seed(base: int, layer: int, pool: int = 0) -> int:
    """Deterministic per-layer payload seed: every holder of a layer has identical bytes
    (with a source pool of P buffers, layer l carries pool buffer l % P)."""
    key = layer % pool if pool > 0 else layer
    h = hashlib.blake2b(f"{base}:{key}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little")


def hist_quantile(hist: List[int], q: float) -> int:
    """Upper edge (us) of the log2 bucket holding quantile q (0 if the histogram is empty)."""
    total = sum(hist)
    if total <= 0:
        return 0
    acc = 0
    for b, n in enumerate(hist):
        acc += n
        if acc >= q * total:
            return 1 << (b + 1)
    return 1 << len(hist)


def mode3_plan(cfg: Config, integer_seconds: bool = True, storage: bool = False) -> "_core.FlowPlan":
    """The mode-3 leader's plan for `cfg` on the TCP data plane, without moving a
    byte: the flow problem Node::schedule_mode3 builds from the announces -
    every node's initial layers as holdings at its Sources rate of their tier
    (disk tier on disk, the others in memory unless `storage`, as `-s` does),
    a demand for every assigned layer its node does not hold (a node that holds
    it in some tier loads it itself: a self-job, node.go:1205-1217), each
    node's NetworkBW as its egress and ingress budget, the config's Links -
    solved by sched/maxflow (reference: flow.go:146-219; with integer_seconds
    T is bisected over whole seconds as the reference does, flow.go:155-187)."""
    holdings: Dict[int, Dict[int, object]] = {}
    size: Dict[int, int] = {}
    for n in cfg.nodes:
        held = holdings.setdefault(n.id, {})
        for st, per in n.initial_layers.items():
            rate = n.sources.get(st, 0)
            on_disk = st == SOURCE_DISK or (storage and st not in (SOURCE_CLIENT, SOURCE_DEVICE))
            loc = (_core.Location.Client if st == SOURCE_CLIENT else _core.Location.Disk if on_disk
                   else _core.Location.Device if st == SOURCE_DEVICE else _core.Location.Inmem)
            for l, sz in per.items():
                held[l] = _core.LayerMeta(loc, rate, _core.SourceType(st), sz)
                size[l] = max(size.get(l, 0), sz)
    demands = [(l, d, size.get(l, cfg.layer_size)) for d, ls in sorted(cfg.assignment.items()) for l in ls
               if l not in holdings.get(d, {})]
    bw = {n.id: n.network_bw for n in cfg.nodes if n.network_bw > 0}
    links = {(s, d): b for s, per in cfg.links.items() for d, b in per.items()}
    return _core.solve_flow(holdings, demands, bw, bw, links=links, integer_seconds=integer_seconds)


def _sig(x: float, digits: int = 4) -> float:
    """`x` to `digits` significant digits (probe rates: GB/s at any fabric scale)."""
    return float(f"{x:.{digits}g}")


@dataclass
class SessionResult:
    ok: bool
    seconds: float  # this rank's wall time for the session (announce -> startup)
    time_to_deliver_s: float = 0.0  # leader: reference "Time to deliver"
    bytes_planned: int = 0
    jobs: int = 0
    plan_ms: float = 0.0
    plan_cached: bool = False
    plan_solver: str = ""  # leader: "mode1:links", "flow", "lp", ...
    plan_gap_bytes: int = 0  # leader, mode 3: bytes the plan left uncovered (invariant: 0)
    plan_sched_ms: float = 0.0  # leader: the scheduler's share of plan_ms (or the plan-cache lookup)
    plan_dispatch_ms: float = 0.0  # leader: encoding + sending the transfer batches
    flow_T: float = 0.0
    error: str = ""
    nacks: int = 0  # leader: chunk re-sends after CRC mismatches
    redispatched: int = 0  # leader: jobs re-sent from another owner after a deadline
    recoveries: int = 0  # leader: communicator shrinks after a rank died (planned engines)
    dropped: int = 0  # leader: (dest, layer) pairs given up (dead dest / no live holder)
    engine_stats: Dict[str, float] = field(default_factory=dict)


class _DeviceBytes:
    """__cuda_array_interface__ of `n` bytes of HBM owned by a Runtime's engine
    (torch.as_tensor keeps this object, and so the Runtime, alive)."""

    def __init__(self, owner, ptr: int, n: int):
        self._owner = owner
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (int(ptr), False),
                                         "version": 3, "strides": None, "stream": None}


class Runtime:
    def __init__(
        self,
        cfg: Config,
        node_id: int,
        *,
        engine: str = "host",
        transport: str = "tcp",
        storage_path: str = "",
        chunk_bytes: int = 64 * MiB,
        verify: bool = True,
        payload_seed: int = 0,
        registry: Optional[Dict[int, str]] = None,
        barrier: Optional[Callable[[], None]] = None,
        nccl_uid: Optional[bytes] = None,
        device: Optional[int] = None,
        listen_addr: Optional[str] = None,
        poison: bool = True,
        sim_key: str = "sim",
        pack: str = "none",
        pack_block: int = 128,
        store: str = "packed",
        inject_corrupt: float = 0.0,
        inject_seed: int = 1,
        max_retries: int = 4,
        group_timeout_s: float = 300.0,
        host_link_rate: Optional[Dict[int, int]] = None,
        group_peers: int = 1,
        persist_dir: str = "",
        engine_opts: Optional[Dict[str, object]] = None,
        source_pool: int = 0,
        node_disk_gbps: float = 0.0,
        node_key: str = "",
        host_share: bool = False,
        host_share_timeout_s: float = 600.0,
        layer_source: Optional[Callable[[int, int], object]] = None,
        hosts: Optional[Dict[int, object]] = None,
    ):
        self.cfg = cfg
        self.node_id = node_id
        self.me = cfg.node(node_id)
        self.is_leader = cfg.leader().id == node_id
        self.engine_kind = engine
        self.storage_path = storage_path
        self.chunk_bytes = cfg.chunk_bytes or chunk_bytes
        if pack not in ("none", "fp8"):
            raise ValueError(f"unknown pack format {pack!r}")
        if pack != "none" and engine not in ("rccl", "sim"):
            raise ValueError("--pack needs the planned (rccl/sim) data engine")
        if store not in ("packed", "bf16"):
            raise ValueError(f"unknown store format {store!r}")
        if store == "bf16" and pack != "fp8":
            raise ValueError("--store bf16 dequantizes fp8-packed layers: it needs --pack fp8")
        self.pack = pack
        self.store = store
        self.pack_block = pack_block
        self.host_link_rate = dict(host_link_rate or {})
        self.persist_dir = persist_dir
        # Host-tier sources share `source_pool` distinct buffers (layer l -> l % P):
        # large presets (126 x 3 GiB bf16) fit host memory; every layer still
        # carries random bytes and its own CRC manifest.
        self.source_pool = int(source_pool)
        self._pool: Dict[int, object] = {}
        # The bytes of the layers this rank seeds: layer_source(layer, size) ->
        # any buffer of `size` bytes (bytes, numpy array, CPU tensor; e.g. a
        # models/weights.py blob). Default: random bytes (splitmix64, layer_seed).
        self.layer_source = layer_source
        if layer_source is not None and self.source_pool:
            raise ValueError("layer_source and source_pool are exclusive (a pool reuses one buffer for many layers)")
        # One NVMe shared by every rank of this node (BASELINE config #4): the
        # disk readers of all ranks draw from one budget (engine/node_pacer.h,
        # keyed by node_key) and mode 3 plans the ranks' disk tiers as one group.
        self.node_disk_gbps = float(node_disk_gbps)
        # Node-shared host tier (BASELINE config #2 from host memory): host-tier
        # layers live in POSIX shared memory created by their holder and mapped
        # (and HIP-registered) by every rank of the node; every rank then holds
        # them as host-tier sources and mode 0 stages one slice per rank.
        self.host_share = bool(host_share)
        self.node_key = node_key or sim_key
        self.host_share_timeout_s = host_share_timeout_s
        self._shared: List[object] = []
        self.shared_mapped: List[int] = []  # layers this rank maps from another rank's shared host tier
        self.verify = verify
        self.payload_seed = payload_seed
        self._barrier = barrier or (lambda: None)
        self.node_ids = sorted(n.id for n in cfg.nodes)
        # node -> host group: GPUs of one host share its xGMI mesh, hosts are
        # joined by one NIC per GPU (config "Host", or `hosts` - e.g. every
        # rank's hostname under a multi-node torchrun - which takes precedence)
        if hosts:
            groups: Dict[object, int] = {}
            self.hosts = {n: groups.setdefault(hosts.get(n, ""), len(groups)) for n in self.node_ids}
        else:
            self.hosts = cfg.hosts()
        self.rank = self.node_ids.index(node_id)
        self.world = len(self.node_ids)
        self.sizes = cfg.layer_sizes()
        if pack == "fp8":
            # fp8 packs whole bf16 scale blocks of every chunk (core/fp8.h layout)
            unit = 2 * pack_block
            bad = {l: s for l, s in self.sizes.items() if s % unit}
            if bad or self.chunk_bytes % unit:
                raise ValueError(f"--pack fp8 needs layer sizes and the chunk size to be multiples of {unit} B "
                                 f"(2 bytes x {pack_block}-element scale blocks); layers {sorted(bad)[:8]} are not")
        self.epoch = 0
        self._closed = False
        self.device: Optional[int] = None
        self.keep: List[object] = []  # buffers that must outlive sessions
        # Closed-loop link rates (planned engines): per peer node, the EWMA of
        # this rank's measured busy throughput on the link to it (sends) and on
        # the link from it (receives), reported with its announce.
        self.link_est: Dict[int, float] = {}      # out: this rank -> peer (B/s)
        self.link_est_in: Dict[int, float] = {}   # in: peer -> this rank (B/s)
        self.link_obs: Dict[tuple, int] = {}      # (dir, peer): sessions that measured the link
        self.link_probe: Dict[int, float] = {}  # pre-flight probe's concurrent send rates (B/s)
        self.link_probe_in: Dict[int, float] = {}  # ... and receive rates (the links into this rank)
        self.link_slow_streak: Dict[tuple, int] = {}  # (dir, peer): observations below LINK_SLOW x the median
        self.link_level: Dict[str, float] = {}  # dir -> the uniform level every normal link reports (B/s)
        self._links0: Optional[Dict[str, Dict[int, float]]] = None
        self.disk_paths: List[str] = []  # this rank's disk-tier layer files

        reg = dict(registry) if registry is not None else cfg.registry()
        if transport == "inproc":
            self.transport = _core.inproc_transport(reg.get(node_id, str(node_id)), reg)
        else:
            addr = listen_addr or reg.get(node_id) or "127.0.0.1:0"
            self.transport = _core.tcp_transport(addr, reg)
            reg[node_id] = self.transport.address()
            self.transport.set_registry(reg)
            # a layer message's sizes come from the wire: nothing larger than this
            # config's largest layer is accepted (tcp.cc receive_layer)
            self.transport.set_max_payload(max([cfg.layer_size, *cfg.layer_sizes().values()]))

        if engine in ("rccl", "sim"):
            pcfg = _core.PlannedConfig()
            pcfg.rank = self.rank
            pcfg.world = self.world
            pcfg.rank_nodes = self.node_ids
            pcfg.chunk_bytes = self.chunk_bytes
            pcfg.verify = verify
            pcfg.poison = poison
            pcfg.pack = 1 if pack == "fp8" else 0
            pcfg.pack_block = pack_block
            pcfg.unpack_store = store == "bf16"
            pcfg.inject_corrupt = inject_corrupt
            pcfg.inject_seed = inject_seed
            pcfg.max_retries = max_retries
            pcfg.group_timeout_s = group_timeout_s
            pcfg.group_peers = group_peers
            pcfg.hosts = self.uniform_hosts()
            if self.node_disk_gbps > 0:
                pcfg.node_disk_rate = int(self.node_disk_gbps * 1e9)
                pcfg.node_disk_key = node_key or sim_key
            # Extra PlannedConfig fields (reserve_cus, nccl_min_ctas, max_inflight_groups, ...).
            for k, v in (engine_opts or {}).items():
                if not hasattr(pcfg, k):
                    raise ValueError(f"unknown planned-engine option {k!r}")
                setattr(pcfg, k, v)
            if engine == "rccl":
                dev = device if device is not None else (self.me.device if self.me.device is not None else 0)
                if self.world > 1 and nccl_uid is None:
                    raise ValueError("rccl engine with world > 1 needs an nccl unique id from the bootstrap")
                _core.set_device(dev)
                self.device = dev
                self.engine = _core.gpu_engine(pcfg, dev, nccl_uid or b"")
            else:
                # Simulated fabric: ranks in this process sharing `sim_key` exchange bytes
                # with RCCL P2P matching semantics (CPU tests of the GPU schedule).
                self.engine = _core.sim_engine(pcfg, sim_key)
        elif engine == "host":
            self.engine = None  # host engines are per session (they bind to one node)
        else:
            raise ValueError(f"unknown engine {engine}")
        # Bytes of each layer in the target tier and on the wire (packed with --pack fp8),
        # and the chunk grid transfers/CRCs run on.
        if self.engine is not None:
            self.slot_sizes = {l: self.engine.slot_size(s) for l, s in self.sizes.items()}
            self.grid = self.engine.chunk_grid
        else:
            self.slot_sizes = dict(self.sizes)
            self.grid = self.chunk_bytes
        self.layers = self._materialize()

    # ---- "device" memory helpers: HIP kernels for rccl, host code for the simulator
    def _dev_fill(self, ptr: int, size: int, seed: int) -> None:
        if self.engine_kind == "rccl":
            _core.fill_random(ptr, size, seed)
            _core.device_synchronize()
        else:
            _core.sim_write(ptr, _core.fill_random_host(size, seed))

    def _dev_crc(self, ptr: int, size: int) -> List[int]:
        if self.engine_kind == "rccl":
            return _core.crc32c_chunks(ptr, size, self.grid)
        return _core.host_crc32c_chunks(ptr, size, self.grid)

    def _source(self, layer: int, size: int) -> memoryview:
        """layer_source's bytes for a layer, checked for size."""
        import torch

        obj = self.layer_source(layer, size)
        if isinstance(obj, torch.Tensor):
            obj = obj.detach().cpu().contiguous().view(torch.uint8).numpy()
        mv = memoryview(obj).cast("B")
        if mv.nbytes != size:
            raise ValueError(f"layer_source({layer}) gave {mv.nbytes} B, the layer is {size} B")
        return mv

    def _source_bytes(self, layer: int, size: int, seed: int, off: int = 0, n: Optional[int] = None) -> bytes:
        n = size - off if n is None else n
        if self.layer_source is not None:
            return bytes(self._source(layer, size)[off:off + n])
        return _core.fill_random_host(n, seed, off) if off else _core.fill_random_host(n, seed)

    def _fill_from_source(self, dev: int, layer: int, size: int, seed: int, host_buf=None) -> None:
        """rccl: the layer's source bytes into device memory `dev` (and `host_buf`)."""
        if self.layer_source is None:
            _core.fill_random(dev, size, seed)
            _core.device_synchronize()
            if host_buf is not None:
                _core.memcpy(host_buf.ptr, dev, size)
            return
        stage = host_buf if host_buf is not None else _core.HostBuffer.malloc(size)
        stage.view()[:] = self._source(layer, size)
        _core.memcpy(dev, stage.ptr, size)

    def _gen_layer(self, layer: int, size: int, seed: int, host_buf=None) -> None:
        """Generate a layer's source bytes (layer_source, or random bf16 bit
        patterns), optionally copy them to `host_buf`, put the target-tier image
        (packed with --pack fp8) into the layer's HBM slot and record its CRC
        manifest."""
        slot = self.engine.device_ptr(layer)
        ssz = self.slot_sizes[layer]
        if self.engine_kind == "rccl":
            if self.pack == "fp8":
                tmp = _core.device_malloc(size)
                try:
                    self._fill_from_source(tmp, layer, size, seed, host_buf)
                    _core.fp8_pack_chunks(tmp, size, self.chunk_bytes, self.pack_block, slot)
                    _core.device_synchronize()
                finally:
                    _core.device_free(tmp)
            else:
                self._fill_from_source(slot, layer, size, seed, host_buf)
        else:
            data = self._source_bytes(layer, size, seed)
            if host_buf is not None:
                _core.sim_write(host_buf.ptr, data)
            if self.pack == "fp8":
                data = _core.fp8_pack_layer_host(data, self.chunk_bytes, self.pack_block)
            _core.sim_write(slot, data)
        self.engine.set_manifest(layer, _core.CrcManifest(self.grid, self._dev_crc(slot, ssz)))

    def _dev_to_host(self, dst: int, src: int, size: int) -> None:
        if self.engine_kind == "rccl":
            _core.memcpy(dst, src, size)
        else:
            _core.sim_write(dst, _core.sim_read(src, size))

    # ------------------------------------------------------------ layers
    def _materialize(self) -> Dict[int, "_core.LayerSrc"]:
        """cmd/config.go:94-198 (CreateLayers / AddClientLayers), MI355X tiers added."""
        layers: Dict[int, _core.LayerSrc] = {}
        gpu = self.engine is not None
        if gpu:
            # Every layer this rank may hold in HBM gets its slot up front.
            want = set(self.cfg.assignment.get(self.node_id, []))
            for per in self.me.initial_layers.values():
                want |= set(per)
            if self.engine_kind == "rccl":
                self._check_hbm_capacity(want)
            for l in sorted(want):
                self.engine.provision(l, self.slot_sizes[l])
        for st, per in sorted(self.me.initial_layers.items()):
            rate = self.me.sources.get(st, 0)
            for l, size in sorted(per.items()):
                seed = layer_seed(self.payload_seed, l, self.source_pool)
                if st == SOURCE_CLIENT:  # metadata only: the node's external client holds the bytes
                    layers[l] = _core.LayerSrc.client(size, rate)
                elif st == SOURCE_DISK or (self.storage_path and st != SOURCE_DEVICE):
                    path = self._disk_layer(l, size, seed)
                    self.disk_paths.append(path)
                    # the file holds the source bytes; the layer's size is its slot size
                    layers[l] = _core.LayerSrc.disk(path, self.slot_sizes[l], rate, _core.SourceType(st))
                    if gpu:
                        self._gen_layer(l, size, seed)
                elif st == SOURCE_DEVICE and gpu:
                    ptr = self.engine.device_ptr(l)
                    self._gen_layer(l, size, seed)
                    self.engine.set_seeded(l, True)
                    layers[l] = _core.layer_src_device(ptr, self.slot_sizes[l])
                elif gpu and self.host_share:
                    buf = _core.HostBuffer.shared(self._hs_name(self.node_id, l), size, True,
                                                  self.engine_kind == "rccl")
                    self._shared.append(buf)
                    self._gen_layer(l, size, seed, host_buf=buf)
                    layers[l] = self._host_src(buf, l, size, rate, st)
                elif gpu:
                    key = (l % self.source_pool, size) if self.source_pool > 0 else None
                    if key is not None and key in self._pool:
                        # shared pool buffer: already holds this residue's bytes
                        buf = self._pool[key]
                        self._gen_layer(l, size, seed)
                    else:
                        buf = (_core.HostBuffer.pinned(size) if self.engine_kind == "rccl"
                               else _core.HostBuffer.malloc(size))
                        self._gen_layer(l, size, seed, host_buf=buf)
                        if key is not None:
                            self._pool[key] = buf
                    layers[l] = self._host_src(buf, l, size, rate, st)
                else:
                    data = self._source_bytes(l, size, seed)
                    layers[l] = _core.LayerSrc.inmem(data, rate, _core.SourceType(st))
        if gpu and self.host_share:
            self._map_shared_layers(layers)
        client = self.cfg.client(self.node_id)
        if client is not None:  # AddClientLayers (config.go:119-131): metadata only
            for l, rate in client.layers.items():
                if l not in layers:
                    layers[l] = _core.LayerSrc.client(self.cfg.layer_size, rate)
        for l, (path, entry) in self._resumable().items():
            if l in layers:
                continue
            # A layer this node received in an earlier run: announce it as a disk-tier
            # copy, so the leader promotes it locally instead of moving it again. A
            # layer persisted in part (chunk-granular resume) is announced as the
            # byte ranges of its chunks; the leader plans only the rest.
            src = _core.LayerSrc.disk(path, self.slot_sizes[l], 0, _core.SourceType.Disk)
            ranges = self._chunk_ranges(entry, self.slot_sizes[l])
            if ranges is not None:
                src.ranges = ranges
                self.resumed_partial.append(l)
            layers[l] = src
            if gpu:
                self.engine.set_manifest(l, _core.CrcManifest(self.grid, entry["crc"]))
                self.engine.set_source_packed(l, True)
            self.resumed.append(l)
        return layers

    def _host_src(self, buf, l: int, size: int, rate: int, st: int):
        src = _core.layer_src_from_buffer(buf, rate, _core.SourceType(st))
        if self.slot_sizes[l] != size:  # packed: bf16 source, fp8 slot
            src.data_size = self.slot_sizes[l]
            meta = src.meta
            meta.size = self.slot_sizes[l]
            src.meta = meta
        return src

    def _hs_name(self, holder: int, layer) -> str:
        return f"dld_hs_{self.node_key}_{holder}_{layer}"

    def _map_shared_layers(self, layers) -> None:
        """host_share: publish this rank's segments (a ready marker), then map every
        other rank's host-tier layers as host-tier sources of this rank - ranks
        of this rank's own host only: another host's /dev/shm is not reachable
        (and with fake host labels, DISSEM_FAKE_HOSTS, it must not be either)."""
        mine = [l for st, per in self.me.initial_layers.items() if st not in (SOURCE_DISK, SOURCE_DEVICE, SOURCE_CLIENT)
                for l in per]
        if mine:
            self._shared.append(_core.HostBuffer.shared(self._hs_name(self.node_id, "ready"), 4096, True, False))
        pin = self.engine_kind == "rccl"
        my_host = self.hosts.get(self.node_id, 0)
        for n in self.cfg.nodes:
            if n.id == self.node_id or self.hosts.get(n.id, 0) != my_host:
                continue
            theirs = [(l, size) for st, per in n.initial_layers.items()
                      if st not in (SOURCE_DISK, SOURCE_DEVICE, SOURCE_CLIENT) for l, size in per.items()]
            if not theirs or self.storage_path:
                continue
            deadline = time.monotonic() + self.host_share_timeout_s
            while not _core.HostBuffer.shared_exists(self._hs_name(n.id, "ready")):
                if time.monotonic() > deadline:
                    raise RuntimeError(f"host_share: node {n.id} did not publish its host layers in "
                                       f"{self.host_share_timeout_s:.0f} s")
                time.sleep(0.02)
            for l, size in theirs:
                if l in layers:
                    continue
                buf = _core.HostBuffer.shared(self._hs_name(n.id, l), size, False, pin)
                self._shared.append(buf)
                layers[l] = self._host_src(buf, l, size, 0, 2)
                self.shared_mapped.append(l)

    def unlink_shared(self) -> None:
        """Remove this rank's shared segment names once every rank has mapped them
        (call after a barrier; mappings stay valid, nothing is left in /dev/shm)."""
        for st, per in self.me.initial_layers.items():
            for l in per:
                _core.HostBuffer.shared_unlink(self._hs_name(self.node_id, l))
        _core.HostBuffer.shared_unlink(self._hs_name(self.node_id, "ready"))

    # Planning estimates for the GPU topology (per direction): one xGMI link as
    # RCCL P2P drives it, and one GPU's PCIe host->HBM staging (57.5 GB/s
    # measured, profiles/r1_h2d/).
    XGMI_PLAN_GBPS = 50.0
    PCIE_PLAN_GBPS = 55.0
    # HBM ingress (write) budget of a GPU for the mode-3 graph: measured HBM copy
    # rate (profiles/r1_fp8/kernel_bench.json: 5.3 TB/s) - never binding next to
    # 7 xGMI links, but the graph states it (SURVEY C13')
    HBM_PLAN_GBPS = 5000.0
    # One GPU's NIC per direction on a multi-node cluster (a 400 Gb/s NIC per
    # GPU): the rate of a link between GPUs of different hosts in the plan.
    NIC_PLAN_GBPS = 50.0

    # Headroom kept free of layer slots: CRC workspaces, fp8 staging scratch,
    # RCCL's own buffers, PyTorch's context.
    HBM_HEADROOM = 4 << 30

    def _check_hbm_capacity(self, layers) -> None:
        """refuse a placement that cannot fit before allocating any of it
        (126 x 3 GiB bf16 = 378 GiB does not fit 288 GB; fp8 packing or a partitioned
        assignment does)."""
        need = sum(self.slot_sizes[l] for l in layers)
        if self.store == "bf16":
            # every layer this rank holds also gets its dequantized bf16 slot
            need += sum(self.sizes[l] for l in layers)
        free, total = _core.mem_info()
        if need + self.HBM_HEADROOM > free:
            raise ValueError(
                f"node {self.node_id}: its {len(layers)} layer slots need {need / 2**30:.1f} GiB of HBM but only "
                f"{free / 2**30:.1f} of {total / 2**30:.1f} GiB are free (keeping {self.HBM_HEADROOM >> 30} GiB "
                f"headroom); use --pack fp8 or an assignment that partitions the layers")

    # ------------------------------------------------------ persist / resume
    PERSIST_MANIFEST = "manifest.json"

    def _persist_root(self) -> str:
        return os.path.join(self.persist_dir, str(self.node_id))

    def _chunk_ranges(self, entry, stored: int):
        """Merged [start, end) byte ranges of a partial entry's chunks (None: whole layer)."""
        chunks = entry.get("chunks")
        n = (stored + self.grid - 1) // self.grid
        if chunks is None or len(set(chunks)) >= n:
            return None
        out = []
        for c in sorted(set(chunks)):
            a, b = c * self.grid, min((c + 1) * self.grid, stored)
            if out and out[-1][1] == a:
                out[-1] = (out[-1][0], b)
            else:
                out.append((a, b))
        return out

    def _resumable(self) -> Dict[int, tuple]:
        """Persisted layers whose file and manifest entry match this run's layout."""
        self.resumed: List[int] = []
        self.resumed_partial: List[int] = []
        if not self.persist_dir:
            return {}
        root = self._persist_root()
        try:
            with open(os.path.join(root, self.PERSIST_MANIFEST)) as f:
                man = json.load(f)
        except (OSError, ValueError):
            return {}
        out = {}
        for lid, e in man.get("layers", {}).items():
            l = int(lid)
            path = os.path.join(root, f"{l}.layer")
            if (l not in self.sizes or e.get("size") != self.sizes[l] or e.get("stored") != self.slot_sizes[l]
                    or e.get("pack") != self.pack or e.get("grid") != self.grid or not os.path.exists(path)
                    or os.path.getsize(path) != e["stored"] or (e.get("chunks") is not None and not e["chunks"])):
                continue
            out[l] = (path, e)
        return out

    def persist(self, layers: Optional[List[int]] = None, partial: bool = False) -> List[int]:
        """Write this node's target-tier layers (default: its assignment) to
        <persist_dir>/<node>/<layer>.layer plus a manifest (size, slot size,
        packing, chunk grid, CRC32C per chunk). SURVEY §5.4; a later run with
        the same --persist-dir announces them as disk-tier layers.

        ``partial`` (planned engines, e.g. after a failed session): also keep
        layers that landed only in part - each verified-resident chunk is
        written at its offset of a sparse layer file and listed under
        "chunks", so the next run receives only the missing chunks."""
        if not self.persist_dir:
            raise ValueError("no persist_dir configured")
        root = self._persist_root()
        os.makedirs(root, exist_ok=True)
        mpath = os.path.join(root, self.PERSIST_MANIFEST)
        try:
            with open(mpath) as f:
                man = json.load(f)
        except (OSError, ValueError):
            man = {"layers": {}}
        todo = layers if layers is not None else list(self.cfg.assignment.get(self.node_id, []))
        done = []
        for l in todo:
            stored = self.slot_sizes[l]
            path = os.path.join(root, f"{l}.layer")
            tmp = path + ".tmp"
            entry = {"size": self.sizes[l], "stored": stored, "pack": self.pack, "grid": self.grid}
            if self.engine is not None:
                ptr = self.engine.device_ptr(l)
                nchunks = (stored + self.grid - 1) // self.grid
                have = list(self.engine.resident_chunks(l)) if partial else list(range(nchunks))
                if not have:
                    continue
                whole = len(have) == nchunks
                crc_all = self._dev_crc(ptr, stored)
                crc = [crc_all[c] if c in set(have) else 0 for c in range(nchunks)]
                step = max(self.grid, 64 * MiB // self.grid * self.grid)
                buf = (_core.HostBuffer.pinned(step) if self.engine_kind == "rccl" else _core.HostBuffer.malloc(step))
                with open(tmp, "wb") as f:
                    f.truncate(stored)  # sparse: chunks that did not land stay holes
                    if whole:
                        for off in range(0, stored, step):
                            n = min(step, stored - off)
                            self._dev_to_host(buf.ptr, ptr + off, n)
                            f.write(buf.view()[:n])
                    else:
                        for c in have:
                            off, n = c * self.grid, min(self.grid, stored - c * self.grid)
                            self._dev_to_host(buf.ptr, ptr + off, n)
                            f.seek(off)
                            f.write(buf.view()[:n])
                if not whole:
                    entry["chunks"] = sorted(have)
            else:
                data = self._last_node.layer(l).host_bytes()
                if not data:
                    continue
                crc = [_core.crc32c(data[o : o + self.grid]) for o in range(0, len(data), self.grid)]
                with open(tmp, "wb") as f:
                    f.write(data)
            entry["crc"] = crc
            os.replace(tmp, path)
            man["layers"][str(l)] = entry
            done.append(l)
        with open(mpath + ".tmp", "w") as f:
            json.dump(man, f)
        os.replace(mpath + ".tmp", mpath)
        return done

    def _disk_layer(self, layer: int, size: int, seed: int) -> str:
        """<s>/layers/<id>/<layer>.layer, written only if missing (config.go:133-157)."""
        root = self.storage_path or os.path.join(os.getcwd(), "storage")
        d = os.path.join(root, "layers", str(self.node_id))
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, f"{layer}.layer")
        if self.layer_source is not None or not os.path.exists(path) or os.path.getsize(path) != size:
            tmp = path + ".tmp"
            with open(tmp, "wb") as f:
                step = 256 * MiB
                for off in range(0, size, step):
                    n = min(step, size - off)
                    f.write(self._source_bytes(layer, size, seed, off, n))
            os.replace(tmp, path)
        return path

    def drop_disk_cache(self) -> float:
        """Write back and evict this rank's disk-tier layer files from the page
        cache (the reference drops every cache before a run, conf/exe.sh:17);
        returns the largest fraction of any file still resident afterwards
        (0.0 = every read of the next session goes to the device; -1: no files)."""
        worst = -1.0
        for p in self.disk_paths:
            worst = max(worst, _core.file_cache_drop(p))
        return worst

    # ---------------------------------------------------------- sessions
    def run(self, mode: int, *, timeout: float = 600.0, **policy) -> SessionResult:
        """prepare() + barrier + execute(): one full dissemination session."""
        self.prepare(mode, **policy)
        self._barrier()  # every rank listens before anyone announces
        return self.execute(timeout)

    def prepare(
        self,
        mode: int,
        *,
        seed: int = 0,
        owner_policy: str = "random",
        pull_window: int = 1,
        relay: bool = True,
        collective: bool = False,
        integer_seconds: bool = False,
        job_timeout_s: float = 0.0,
        job_min_rate: float = 0.0,
        pull_job_bytes: int = 0,
        xgmi_link_gbps: Optional[float] = None,
        stage_gbps: Optional[float] = None,
        link_bw: Optional[Dict[tuple, int]] = None,
        hbm_gbps: Optional[float] = None,
        adapt_links: bool = True,
        hierarchical: bool = True,
        nic_gbps: Optional[float] = None,
    ) -> None:
        """Reset the data plane and start a fresh Node for the next epoch (untimed).

        On the rccl engine the planners see the GPU topology by default: every
        directed pair of GPUs as a link of ``xgmi_link_gbps`` (divided by its hop
        count; default XGMI_PLAN_GBPS) and every GPU's host->HBM staging at
        ``stage_gbps`` (default PCIE_PLAN_GBPS). ``link_bw`` overrides both the
        config's Links and the probe (e.g. per-link rates measured in an earlier
        session). ``hbm_gbps`` is every GPU's HBM ingress budget in the mode-3
        graph (default HBM_PLAN_GBPS on rccl, unlimited elsewhere).

        ``adapt_links`` (closed loop): this rank announces its measured send
        rate to each peer (``link_report``: EWMA over earlier sessions and the
        pre-flight probe), and the leader plans on every rank's reports in place
        of the estimates above.

        ``hierarchical`` (multi-host runs): mode 1's "links" policy imports a
        layer once per host and relays it over that host's xGMI mesh
        (Node::schedule_imports), and mode 0's relay broadcast runs as a
        three-level tree (Node::relay_across_hosts), and mode 3 budgets each
        node's traffic to other hosts by its NIC (``nic_gbps``, default
        NIC_PLAN_GBPS); False plans as on one host."""
        self.epoch += 1
        if self.engine is not None:
            self.engine.reset_session()
            self._stats0 = self._engine_stats()
            self._links0 = self.link_stats()
        nc = _core.NodeConfig()
        nc.id = self.node_id
        nc.leader = self.cfg.leader().id
        nc.mode = mode
        nc.epoch = self.epoch
        nc.seed = seed
        nc.owner_policy = owner_policy
        nc.pull_window = pull_window
        nc.relay = relay
        nc.collective = collective
        nc.network_bw = {k: v for k, v in self.cfg.network_bw().items()}
        nc.link_bw = {(s, d): bw for s, per in self.cfg.links.items() for d, bw in per.items()}
        gpu = self.engine_kind == "rccl"
        if xgmi_link_gbps is None:
            xgmi_link_gbps = self.XGMI_PLAN_GBPS if gpu else 0.0
        if stage_gbps is None:
            stage_gbps = self.PCIE_PLAN_GBPS if gpu else 0.0
        if not nc.link_bw and xgmi_link_gbps > 0 and gpu:
            nc.link_bw = self.topology_link_bw(xgmi_link_gbps)
        if link_bw:
            nc.link_bw = dict(link_bw)
        if stage_gbps > 0:
            nc.stage_bw = {n.id: int(stage_gbps * 1e9) for n in self.cfg.nodes}
        if hbm_gbps is None:
            hbm_gbps = self.HBM_PLAN_GBPS if gpu else 0.0
        if hbm_gbps > 0:
            nc.hbm_bw = {n.id: int(hbm_gbps * 1e9) for n in self.cfg.nodes}
        nc.host_share = self.host_share
        if hierarchical and len(set(self.hosts.values())) > 1:
            nc.host = dict(self.hosts)
            # mode 3 budgets every node's traffic to other hosts by its NIC
            nc.nic_bw = {n: int((nic_gbps if nic_gbps is not None else self.NIC_PLAN_GBPS) * 1e9)
                         for n in self.node_ids}
        if self.node_disk_gbps > 0:  # every rank of a host reads that host's one NVMe
            nc.disk_group = {n.id: self.hosts.get(n.id, 0) for n in self.cfg.nodes}
            nc.disk_group_bw = {h: int(self.node_disk_gbps * 1e9) for h in set(self.hosts.values())}
        nc.adapt_links = adapt_links
        if adapt_links:
            nc.link_report = self.link_report()
            nc.link_report_in = self.link_report_in()
        nc.integer_seconds = integer_seconds
        nc.job_timeout_s = job_timeout_s
        nc.job_min_rate = job_min_rate
        nc.pull_job_bytes = pull_job_bytes
        nc.range_acks = mode == 2 and pull_job_bytes > 0
        nc.align = self.grid if self.engine is not None else 1
        eng = self.engine if self.engine is not None else _core.host_engine(self.host_link_rate)
        assign = {k: v for k, v in self.cfg.assignment.items()} if self.is_leader else {}
        node = _core.Node(nc, self.transport, eng, self.layers, assign, self.is_leader)
        node.start()
        self._node = node

    def execute(self, timeout: float = 600.0, announce_retry_s: float = 0.0) -> SessionResult:
        """Announce, then block until Ready (leader: assignment satisfied; receiver: startup).

        ``announce_retry_s`` retries the announce while the leader is not listening yet
        (separately launched processes); the reference fails on the first dial error.
        """
        node = self._node
        t0 = _core.vclock_now()  # the steady clock; model time in a virtual-clock simulation
        if not self.is_leader:
            deadline = time.monotonic() + announce_retry_s
            while True:
                try:
                    node.announce()
                    break
                except RuntimeError:
                    if time.monotonic() >= deadline:
                        raise
                    time.sleep(0.1)
        ok = node.wait_ready(timeout)
        t1 = _core.vclock_now()
        err = ""
        if self.engine is not None:
            err = self.engine.error()
            if err:
                ok = False
        st = node.stats()
        res = SessionResult(
            ok=ok,
            seconds=t1 - t0,
            time_to_deliver_s=st.time_to_deliver_s,
            bytes_planned=st.bytes_planned,
            jobs=st.jobs_dispatched,
            plan_ms=st.plan_ms,
            plan_cached=st.plan_cached,
            plan_solver=st.plan_solver,
            plan_gap_bytes=st.plan_gap_bytes,
            plan_sched_ms=st.plan_sched_ms,
            plan_dispatch_ms=st.plan_dispatch_ms,
            flow_T=st.flow_T,
            error=err if err else ("" if ok else "timeout waiting for Ready()"),
            nacks=st.nacks,
            redispatched=st.redispatched,
            recoveries=st.recoveries,
            dropped=st.dropped,
        )
        if self.engine is not None and ok:
            self.engine.quiesce()  # trailing verifications of chunks nobody waited for
            now = self._engine_stats()
            res.engine_stats = {k: now[k] - self._stats0.get(k, 0) for k in now if not k.endswith("_hist")}
            for h in ("group_us_hist", "land_us_hist"):
                delta = [a - b for a, b in zip(now[h], self._stats0[h])]
                for q in (0.5, 0.99):
                    res.engine_stats[f"{h[:-8]}_p{int(q * 100)}_us"] = hist_quantile(delta, q)
        if self.engine is not None and ok:
            self._observe_session_links()
        if ok:
            node.stop()
        self._last_node = node  # on failure keep it alive for inspection
        return res

    def uniform_hosts(self) -> int:
        """H when the ranks fill H hosts with the same number of GPUs each, in
        rank order (torchrun's layout; the engine's host-aware comm lanes,
        backend.h host_lanes), else 1."""
        seq = [self.hosts.get(n, 0) for n in self.node_ids]
        h = len(set(seq))
        if h <= 1 or self.world % h:
            return 1
        g = self.world // h
        blocks = [seq[i * g:(i + 1) * g] for i in range(h)]
        if any(len(set(b)) != 1 for b in blocks) or len({b[0] for b in blocks}) != h:
            return 1
        return h

    # ------------------------------------------------- closed-loop link rates
    # Per directed link touching this rank, a CAPACITY estimate from earlier
    # sessions: bytes over the device time of the P2P groups that carried them,
    # timed at this end - sends for the links out of this rank, receives for
    # the links into it (EWMA over sessions). Either end's time includes
    # waiting for the other end to post (an RCCL send kernel spins until its
    # receive is posted, and a receive until its send is), so the leader plans
    # each link on the FASTER of its two ends' reports (Node::merge_link_rates):
    # the later poster timed the transfer alone. A receiver that posts late
    # slows the send-side reading of the links into it, never the plan.
    # The pre-flight probe (both ends posted together) floors a send-side
    # estimate until LINK_PROBE_SESSIONS sessions have measured the link;
    # from then on the sessions alone decide, so a link that degrades after
    # the probe is seen. The report the leader plans on is uniform unless a
    # link is really slower than the others:
    #   * every normal link reports the same level U (the median capacity of
    #     its direction, moved only when the median moves by more than
    #     LINK_LEVEL_HYST), so a uniform mesh plans uniformly and identically
    #     session after session (the leader's plan cache then replays it);
    #   * a link whose capacity stayed below LINK_SLOW x the median in
    #     LINK_SLOW_SESSIONS consecutive observations (the probe counts as one)
    #     reports its own capacity, and the plans route around it.
    # Reference analog: node.go:774-793 times jobs, :1044-1053 steers by them.
    LINK_EWMA_ALPHA = 0.5   # weight of the newest measurement
    LINK_SLOW = 0.7         # a link below this fraction of the median capacity ...
    LINK_SLOW_SESSIONS = 2  # ... in this many consecutive observations is planned at its own rate
    LINK_LEVEL_HYST = 0.10  # the uniform level follows the median only past this relative change
    LINK_MIN_CHUNKS = 4     # a link must have carried this many grid chunks in a session to be measured
    LINK_PROBE_SESSIONS = 2  # sessions after which the probe no longer floors a link

    def _est(self, d: str) -> Dict[int, float]:
        return self.link_est if d == "out" else self.link_est_in

    def observe_links(self, rates: Dict[int, float], rates_in: Optional[Dict[int, float]] = None) -> None:
        """Fold one session's measured rates (peer node -> B/s; send side, and
        optionally receive side) into the per-link EWMAs."""
        a = self.LINK_EWMA_ALPHA
        for d, rs in (("out", rates), ("in", rates_in or {})):
            est = self._est(d)
            for p, r in rs.items():
                if r is None or r <= 0 or p == self.node_id:
                    continue
                old = est.get(p)
                est[p] = float(r) if old is None else old + a * (float(r) - old)
                self.link_obs[(d, p)] = self.link_obs.get((d, p), 0) + 1
            if rs:
                self._update_link_state(d)

    def observe_probe(self, rates: Dict[int, float], rates_in: Optional[Dict[int, float]] = None) -> None:
        """The pre-flight probe's concurrent rates (peer node -> B/s) at this
        rank's sending end and, optionally, its receiving end: the floor of
        every link's capacity until sessions measured it."""
        for d, rs in (("out", rates), ("in", rates_in or {})):
            probe = self.link_probe if d == "out" else self.link_probe_in
            for p, r in rs.items():
                if r and r > 0 and p != self.node_id:
                    probe[p] = float(r)
            if rs:
                self._update_link_state(d)

    def link_capacity(self, d: str = "out") -> Dict[int, float]:
        """Per peer node (B/s): the session EWMA of direction `d`, floored by the
        probe while fewer than LINK_PROBE_SESSIONS sessions measured the link
        (the probe alone before any)."""
        est = self._est(d)
        probe = self.link_probe if d == "out" else self.link_probe_in
        out = {}
        for p in set(est) | set(probe):
            e = est.get(p, 0.0)
            if p in probe and self.link_obs.get((d, p), 0) < self.LINK_PROBE_SESSIONS:
                e = max(e, probe[p])
            out[p] = e
        return out

    def _update_link_state(self, d: str) -> None:
        cap = self.link_capacity(d)
        if not cap:
            return
        vals = sorted(cap.values())
        med = vals[len(vals) // 2]
        for p, c in cap.items():
            k = (d, p)
            self.link_slow_streak[k] = self.link_slow_streak.get(k, 0) + 1 if c < self.LINK_SLOW * med else 0
        lvl = self.link_level.get(d)
        if lvl is None or abs(med - lvl) > self.LINK_LEVEL_HYST * lvl:
            self.link_level[d] = med

    def _observe_session_links(self) -> None:
        """After a session: this rank's bytes to / from each peer over the device
        time of the P2P groups that carried them (per directed link busy throughput)."""
        if self._links0 is None:
            return
        now = self.link_stats()
        got = {}
        for d, bytes_k, ms_k in (("out", "sent", "send_busy_ms"), ("in", "recv", "recv_busy_ms")):
            rates = {}
            for p, b in now[bytes_k].items():
                db = b - self._links0[bytes_k].get(p, 0)
                dms = now[ms_k].get(p, 0.0) - self._links0[ms_k].get(p, 0.0)
                if db >= self.LINK_MIN_CHUNKS * self.grid and dms > 0:
                    rates[self.node_ids[p]] = db / (dms / 1e3)
            got[d] = rates
        if got["out"] or got["in"]:
            self.observe_links(got["out"], got["in"])

    def _report(self, d: str) -> Dict[int, int]:
        cap = self.link_capacity(d)
        lvl = self.link_level.get(d)
        if not cap or lvl is None:
            return {}
        return {p: int(c if self.link_slow_streak.get((d, p), 0) >= self.LINK_SLOW_SESSIONS else lvl)
                for p, c in cap.items()}

    def link_report(self) -> Dict[int, int]:
        """What this rank announces for its links out (B/s per peer node): the
        uniform level, or a persistently slow link's own capacity (see above)."""
        return self._report("out")

    def link_report_in(self) -> Dict[int, int]:
        """The same for the links into this rank, timed at the receiving end."""
        return self._report("in")

    def plan_link_bw(self) -> Dict[tuple, int]:
        """Leader: the per directed link rates (B/s) its last plan used."""
        node = getattr(self, "_last_node", None) or getattr(self, "_node", None)
        return dict(node.plan_link_bw()) if node is not None and self.is_leader else {}

    def _engine_stats(self) -> Dict[str, float]:
        es = self.engine.stats()
        return {
            k: getattr(es, k)
            for k in ("bytes_sent", "bytes_recv", "bytes_staged", "bytes_verified", "groups", "pieces",
                      "verify_failures", "unverified_pieces", "nacks", "injected", "issue_ms",
                      "suspects", "shrinks", "aborted_pieces", "paced", "order_violations", "disk_wait_ms",
                      "disk_direct_bytes", "disk_buffered_bytes", "scratch_landings", "scratch_buffers",
                      "group_us_hist", "land_us_hist", "verify_busy_ms", "verify_calls", "verify_chunks")
        }

    def topology_link_bw(self, xgmi_gbps: float, pcie_gbps: float = 25.0,
                         nic_gbps: Optional[float] = None) -> Dict[tuple, int]:
        """Per directed (node, node) link capacity for the planners from the GPU
        topology (SURVEY C4/C13'): xGMI links at `xgmi_gbps` divided by their
        hop count, other same-host pairs at `pcie_gbps`, pairs on different
        hosts at `nic_gbps` (default NIC_PLAN_GBPS). Node i runs on device
        `device` from the config, else its index among its host's nodes (one
        process per GPU; this host's topology stands for every host's)."""
        nic = self.NIC_PLAN_GBPS if nic_gbps is None else nic_gbps
        local: Dict[int, int] = {}
        per_host: Dict[int, int] = {}
        for n in self.node_ids:
            h = self.hosts.get(n, 0)
            local[n] = per_host.get(h, 0)
            per_host[h] = local[n] + 1
        dev = {n.id: (n.device if n.device is not None else local[n.id]) for n in self.cfg.nodes}
        links = {(i, j): (kind, hops) for i, j, kind, hops, _ in _core.gpu_topology()}
        out = {}
        for a in self.node_ids:
            for b in self.node_ids:
                if a == b:
                    continue
                if self.hosts.get(a, 0) != self.hosts.get(b, 0):
                    out[(a, b)] = int(nic * 1e9)
                    continue
                kind, hops = links.get((dev[a], dev[b]), ("other", 1))
                gbps = xgmi_gbps / max(1, hops) if kind == "xgmi" else pcie_gbps
                out[(a, b)] = int(gbps * 1e9)
        return out

    def probe_links(self, nbytes: int = 256 * MiB, timeout_s: float = 30.0, solo: bool = True) -> Dict[str, object]:
        """Untimed pre-flight probe of every directed link (planned engines, world > 1).

        ``concurrent``: this rank sends ``nbytes`` to every peer and receives
        ``nbytes`` from every peer at once, each transfer on its directed pair's
        comm lane - the lane set a session drives. ``solo``: then every directed
        pair once more on its own (barrier between pairs; ranks not in the pair
        idle), which separates a slow link from a congested one. Every rank
        calls this at the same time. Rates are this rank's sends (GB/s of device
        time, keyed by peer node); ``concurrent_in`` its receives (the links
        into it, keyed by the sending node). A lane that does not complete within
        ``timeout_s`` raises RuntimeError naming the lane and the pair."""
        if self.engine is None or self.world < 2:
            return {}
        me = self.rank
        peers = [r for r in range(self.world) if r != me]

        def run(ops, what):
            got = self.engine.probe(ops, timeout_s)
            stalled = [o for o in got if not o["done"]]
            if stalled:
                desc = ", ".join(f"lane {o['lane']} ({'send to' if o['send'] else 'recv from'} node "
                                 f"{self.node_ids[o['peer']]})" for o in stalled)
                raise RuntimeError(f"link probe ({what}) stalled after {timeout_s:.0f} s on node {self.node_id}: {desc}")
            return got

        t0 = _core.vclock_now()
        self._barrier()
        got = run([(p, True, nbytes) for p in peers] + [(p, False, nbytes) for p in peers], "concurrent")
        self._barrier()
        conc_ms = (_core.vclock_now() - t0) * 1e3
        out: Dict[str, object] = {
            "bytes": nbytes,
            "concurrent": {self.node_ids[o["peer"]]: _sig(nbytes / (o["ms"] / 1e3) / 1e9) if o["ms"] > 0 else None
                           for o in got if o["send"]},
            # the same pass timed at the receiving end: the links into this rank
            "concurrent_in": {self.node_ids[o["peer"]]: _sig(nbytes / (o["ms"] / 1e3) / 1e9) if o["ms"] > 0 else None
                              for o in got if not o["send"]},
            "concurrent_wall_ms": round(conc_ms, 3),
        }
        if solo:
            rates = {}
            for a in range(self.world):
                for b in range(self.world):
                    if a == b:
                        continue
                    self._barrier()
                    if me == a:
                        o = run([(b, True, nbytes)], f"solo {self.node_ids[a]}->{self.node_ids[b]}")[0]
                        rates[self.node_ids[b]] = _sig(nbytes / (o["ms"] / 1e3) / 1e9) if o["ms"] > 0 else None
                    elif me == b:
                        run([(a, False, nbytes)], f"solo {self.node_ids[a]}->{self.node_ids[b]}")
            self._barrier()
            out["solo"] = rates
        out["probe_ms"] = round((_core.vclock_now() - t0) * 1e3, 1)
        return out

    def link_bytes(self) -> Dict[str, Dict[int, int]]:
        """Cumulative bytes this rank sent to / received from each peer rank (per-link counters)."""
        es = self.engine.stats()
        return {"sent": dict(es.peer_sent), "recv": dict(es.peer_recv)}

    def link_stats(self) -> Dict[str, Dict[int, float]]:
        """Cumulative per-peer counters: bytes sent/received and the device time (ms)
        of the P2P groups that involved the peer; per-lane device time."""
        es = self.engine.stats()
        return {"sent": dict(es.peer_sent), "recv": dict(es.peer_recv), "busy_ms": dict(es.peer_busy_ms),
                "send_busy_ms": dict(es.peer_send_busy_ms), "recv_busy_ms": dict(es.peer_recv_busy_ms),
                "lane_busy_ms": list(es.lane_busy_ms)}

    def layer_bytes(self, layer: int) -> bytes:
        """Bytes of a layer in this rank's target tier (packed with --pack fp8)."""
        if self.engine is not None:
            ptr = self.engine.device_ptr(layer)
            n = self.slot_sizes[layer]
            if self.engine_kind == "sim":
                return _core.sim_read(ptr, n)
            buf = _core.HostBuffer.malloc(n)
            _core.memcpy(buf.ptr, ptr, n)
            return buf.bytes()
        src = self._last_node.layer(layer)
        return src.host_bytes() if src is not None else b""

    def unpacked_layer_bytes(self, layer: int) -> bytes:
        """A packed layer dequantized back to bf16 after checking every packed chunk
        against the manifest (rccl: the fused verify+unpack kernel, one pass over HBM)."""
        if self.pack != "fp8":
            return self.layer_bytes(layer)
        size = self.sizes[layer]
        if self.store == "bf16":
            # already dequantized on the data path (fused verify+unpack per resident chunk)
            out = self.engine.unpacked_ptr(layer)
            if not out:
                raise RuntimeError(f"layer {layer} has no bf16 image (not resident here)")
            if self.engine_kind == "sim":
                return _core.sim_read(out, size)
            buf = _core.HostBuffer.malloc(size)
            _core.memcpy(buf.ptr, out, size)
            return buf.bytes()
        ptr = self.engine.device_ptr(layer)
        if self.engine_kind == "sim":
            packed = _core.sim_read(ptr, self.slot_sizes[layer])
            got = _core.host_crc32c_chunks(ptr, self.slot_sizes[layer], self.grid)
            out = _core.fp8_unpack_layer_host(packed, size, self.chunk_bytes, self.pack_block)
        else:
            dev = _core.device_malloc(size)
            try:
                got = _core.fp8_verify_unpack(ptr, size, self.chunk_bytes, self.pack_block, dev)
                buf = _core.HostBuffer.malloc(size)
                _core.memcpy(buf.ptr, dev, size)
                out = buf.bytes()
            finally:
                _core.device_free(dev)
        want = self.engine.manifest().get(layer)
        if want is not None and list(got) != list(want.crc):
            raise RuntimeError(f"layer {layer}: packed chunks do not match the CRC manifest")
        return out

    # ------------------------------------------------------ serving views
    def layer_tensor(self, layer: int, unpacked: bool = False):
        """The layer as this rank holds it in HBM, as a uint8 torch tensor.

        rccl engine: a zero-copy view of the layer's HBM slot (the packed image
        with --pack fp8; ``unpacked=True`` with --store bf16: the dequantized bf16
        image the fused verify+unpack wrote), valid until close(). The view keeps
        this Runtime alive. Other engines: a CPU copy of the same bytes."""
        import torch

        if self.engine is None:
            return torch.frombuffer(bytearray(self.layer_bytes(layer)), dtype=torch.uint8)
        if unpacked and self.pack == "fp8":
            if self.store != "bf16":
                raise ValueError("unpacked views need --store bf16 (use unpacked_layer_bytes for a copy)")
            ptr, n = self.engine.unpacked_ptr(layer), self.sizes[layer]
        else:
            ptr, n = self.engine.device_ptr(layer), self.slot_sizes[layer]
        if not ptr:
            raise RuntimeError(f"layer {layer} is not resident on rank {self.rank}")
        if self.engine_kind == "sim":
            return torch.frombuffer(bytearray(_core.sim_read(ptr, n)), dtype=torch.uint8)
        if self._closed:
            raise RuntimeError("runtime is closed")
        dev = torch.device("cuda", self.device)
        return torch.as_tensor(_DeviceBytes(self, ptr, n), device=dev)

    def layer_params(self, layer: int, spec):
        """Named bf16 parameter views of a layer that holds a models/weights.py
        blob: zero-copy in HBM on the rccl engine (the dequantized image with
        --pack fp8 --store bf16), CPU copies otherwise."""
        from ..models.weights import unflatten

        if self.pack == "fp8" and self.store != "bf16":
            import torch

            return unflatten(torch.frombuffer(bytearray(self.unpacked_layer_bytes(layer)), dtype=torch.uint8), spec)
        return unflatten(self.layer_tensor(layer, unpacked=True), spec)

    def close(self) -> None:
        self._closed = True
        if self.engine is not None:
            self.engine.shutdown()
        self.transport.close()
        self._shared.clear()  # unmaps (and unlinks the names this rank created)
