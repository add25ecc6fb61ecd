"""Multi-rank GPU schedules on the simulated fabric (CPU).

The planned engine (the MI355X data plane) runs here on SimBackend: host memory
as "HBM", worker threads as the comm/copy/verify queues, and an in-process
fabric with RCCL point-to-point matching (FIFO per directed pair, a group holds
its queue until every op is matched). Everything above the backend - leader
batching, sequence numbers, piece order, group formation, staging deps, CRC
verification, Landed/ack flow - is the same code that drives RCCL on the GPU,
so these tests check the 2/4/8-rank schedules (and their deadlock freedom)
without GPUs. Bytes are verified end to end.
"""

import itertools
import threading

import pytest

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.models.catalog import delivered_bytes, make_workload
from distributed_llm_dissemination_amd.parallel.runtime import Runtime, layer_seed

MiB = 1 << 20
_keys = itertools.count()


def expected_image(rt, layer, size):
    """The layer's bytes in the target tier: the source, or its fp8-packed form."""
    data = _core.fill_random_host(size, layer_seed(0, layer, rt.source_pool))
    if rt.pack == "fp8":
        return _core.fp8_pack_layer_host(data, rt.chunk_bytes, rt.pack_block)
    return data


def run_cluster(cfg, mode, sessions=1, chunk=MiB, rt_kw=None, inspect=None, **policy):
    key = f"sim{next(_keys)}"
    n = len(cfg.nodes)
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=chunk, sim_key=key,
                   **(rt_kw or {})) for i in range(n)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        out = []
        for _ in range(sessions):
            for r in rts:
                r.prepare(mode, **policy)
            res = [None] * n

            def go(i):
                res[i] = rts[i].execute(30)

            ths = [threading.Thread(target=go, args=(i,)) for i in range(n)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            assert all(x.ok for x in res), [x.error for x in res]
            sizes = cfg.layer_sizes()
            for i, r in enumerate(rts):
                for l in cfg.assignment.get(i, []):
                    assert r.layer_bytes(l) == expected_image(r, l, sizes[l]), (i, l)
            out.append(res)
        if inspect is not None:
            inspect(rts)
        return out, key
    finally:
        for r in rts:
            r.close()


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_replicate_random_seeding(n, mode):
    cfg = make_workload(n, 8, 3 * MiB + 4096, tier="host", seeding="random", chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, mode, pull_window=max(1, n - 1))
    leader = res[0]
    assert leader.bytes_planned == delivered_bytes(cfg)
    assert leader.engine_stats["verify_failures"] == 0


@pytest.mark.parametrize("mode,tier", [(0, "host"), (1, "host"), (2, "host"), (3, "host"), (1, "disk")])
def test_layer_sizes_not_multiples_of_16(mode, tier, tmp_path):
    """Layers of any byte size (the reference's experiment layers are
    10,930,691,768 B): every layer's last chunk has an odd length, and the split
    of chunks over owners, relays and mode-3 ranges still delivers every byte."""
    cfg = make_workload(4, 6, 3 * MiB + 13, tier=tier, seeding="random" if mode else "leader", chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, mode, rt_kw={"storage_path": str(tmp_path)}, pull_window=3)
    assert res[0].bytes_planned == delivered_bytes(cfg)
    assert res[0].engine_stats["verify_failures"] == 0


@pytest.mark.parametrize("n", [3, 8])
@pytest.mark.parametrize("relay", [True, False])
def test_mode0_broadcast_relay(n, relay):
    cfg = make_workload(n, 4, 4 * MiB, tier="host", seeding="leader", chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, 0, relay=relay)
    moved = _core.sim_fabric_bytes(key)
    assert moved == (n - 1) * 4 * 4 * MiB  # relay moves the same bytes, spread over all links


def test_mode0_relay_rotates_leftover_chunks():
    """Relay broadcast at 8 ranks: a 16-chunk layer splits 3+3+2+2+2+2+2 over 7
    dests; which dests take the extra chunk rotates from layer to layer, so over
    14 layers every dest's slice - and each of its 6 relay links - carries the
    same 32 chunks (a fixed choice: 42 on two dests, 28 on the rest)."""
    n, L = 8, 14
    cfg = make_workload(n, L, 16 * MiB, tier="host", seeding="leader", chunk_bytes=MiB)
    got = {}
    run_cluster(cfg, 0, relay=True, inspect=lambda rts: got.update(rts[0].link_stats()["sent"]))
    assert sorted(got.values()) == [32 * MiB] * (n - 1), got


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("tier", ["host", "device"])
def test_mode0_collective_broadcast(n, tier):
    """--bcast collective: one ncclBroadcast per chunk rooted at the leader; every
    rank takes part and the receivers verify each chunk."""
    cfg = make_workload(n, 3, 3 * MiB + 4096, tier=tier, seeding="leader", chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, 0, collective=True)
    assert _core.sim_fabric_bytes(key) == (n - 1) * 3 * (3 * MiB + 4096)
    assert sum(r.engine_stats["bytes_verified"] for r in res[1:]) > 0
    if n >= 3:  # one collective piece per chunk of each layer on every rank
        assert all(r.engine_stats["pieces"] == 3 * 4 for r in res)


def test_mode0_collective_falls_back_when_not_everyone_needs_it():
    cfg = make_workload(4, 4, 2 * MiB, tier="host", seeding="leader", assignment="pipeline", chunk_bytes=MiB)
    run_cluster(cfg, 0, collective=True)


@pytest.mark.parametrize("policy", ["random", "balanced", "links"])
def test_mode1_owner_policies_with_copies(policy):
    cfg = make_workload(6, 12, 2 * MiB, tier="host", seeding="uniform", copies=3, seed=5, chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, 1, owner_policy=policy)
    need = sum(1 for r in range(6) for l in range(12) if r not in _owners(cfg, l))
    assert _core.sim_fabric_bytes(key) == need * 2 * MiB


def test_device_seeded_uneven_copies_mode1():
    cfg = make_workload(4, 12, 2 * MiB, tier="device", seeding="uniform", copies=2, seed=3, chunk_bytes=MiB)
    run_cluster(cfg, 1)


def test_pipeline_assignment_mode2_dynamic_batches():
    cfg = make_workload(4, 16, MiB + 512, tier="host", seeding="random", assignment="pipeline", chunk_bytes=MiB)
    run_cluster(cfg, 2, pull_window=1)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_mode2_range_jobs(n):
    """Mode-2 jobs of one chunk each (--pull-job-mib): stealing works inside a
    layer; receivers' range acks retire the jobs."""
    cfg = make_workload(n, 5, 4 * MiB + 4096, tier="host", seeding="random", copies=2, chunk_bytes=MiB)
    (res,), _ = run_cluster(cfg, 2, pull_window=2, pull_job_bytes=MiB)
    assert res[0].jobs > 5 * (n - 2)  # more jobs than (layer, dest) pairs: layers were split


@pytest.mark.parametrize("n", [2, 4])
def test_mode2_dest_holding_a_layer_loads_it_itself(n):
    """Every rank holds every layer (copies = n): mode 2 makes each dest load
    its own copy first (min_loaded_sender), and an idle peer may steal such a
    job as the reference allows (node.go:1036-1042). A rank whose chunk is
    both staged here (for its own sends or load) and sent by a peer keeps one
    writer per byte: the peer's copy lands in scratch (scratch_landings).
    Every byte arrives (run_cluster compares every layer), every byte sent is
    received, each chunk is held once per rank, and no send ever waits on a
    larger-key recv."""
    cfg = make_workload(n, 6, 4 * MiB, tier="host", seeding="random", copies=n, chunk_bytes=MiB)
    outs, _ = run_cluster(cfg, 2, sessions=4, pull_window=2, pull_job_bytes=MiB)
    assert sum(r.engine_stats["order_violations"] for res in outs for r in res) == 0
    for res in outs:
        assert sum(r.engine_stats["bytes_sent"] for r in res) == sum(r.engine_stats["bytes_recv"] for r in res)
        for r in res:  # staged or received - a scratch landing is a received duplicate of a staged chunk
            held = r.engine_stats["bytes_staged"] + r.engine_stats["bytes_recv"] - r.engine_stats["scratch_landings"] * MiB
            assert held == 6 * 4 * MiB, r.engine_stats
    # scratch buffers come from a pool: allocated when all are busy, never one per landing (a free per
    # landing synchronized the GPU under live RCCL groups and hung a recovery, profiles/r6_insure)
    for i in range(n):
        landings = sum(res[i].engine_stats["scratch_landings"] for res in outs)
        allocated = sum(res[i].engine_stats["scratch_buffers"] for res in outs)
        assert allocated <= landings
        if landings >= 4:
            assert allocated < landings, (landings, allocated)


def test_repeated_sessions_reset_state():
    cfg = make_workload(4, 6, 2 * MiB, tier="host", chunk_bytes=MiB)
    outs, _ = run_cluster(cfg, 1, sessions=3)
    assert len(outs) == 3


def test_ranges_not_aligned_to_chunks_mode3():
    # Chunk grid 1 MiB, layer 2.5 MiB: pieces of partial chunks are still exact.
    cfg = make_workload(3, 3, 2 * MiB + MiB // 2, tier="host", seeding="random", copies=2, chunk_bytes=MiB)
    run_cluster(cfg, 3)


def test_disk_tier_staging_through_bounce_ring(tmp_path):
    """BASELINE config #4 shape on the simulator: layers on disk, staged disk ->
    page-aligned bounce ring -> device by reader threads, then P2P + verify."""
    cfg = make_workload(4, 6, 3 * MiB + 8192, tier="disk", seeding="random", chunk_bytes=MiB)
    key = f"sim{next(_keys)}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key,
                   storage_path=str(tmp_path)) for i in range(4)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for _ in range(2):
            for r in rts:
                r.prepare(1)
            res = [None] * 4
            ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(30))) for i in range(4)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            assert all(x.ok for x in res), [x.error for x in res]
            for i, r in enumerate(rts):
                for l in range(6):
                    assert r.layer_bytes(l) == _core.fill_random_host(3 * MiB + 8192, layer_seed(0, l))
    finally:
        for r in rts:
            r.close()


# ---------------------------------------------------------------- fp8 wire/storage format


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("tier", ["host", "device"])
def test_fp8_packed_replication(mode, tier):
    """BASELINE config #5 shape: bf16 sources are packed to fp8 at staging; HBM
    slots, P2P transfers and CRCs all run on the packed chunk grid, so the wire
    carries ~0.53x the bf16 bytes."""
    n, L, size = 4, 6, 3 * MiB + 4096
    cfg = make_workload(n, L, size, tier=tier, seeding="random", chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, mode, rt_kw={"pack": "fp8"}, pull_window=n - 1)
    packed = _core.fp8_packed_size(size, MiB, 128)
    assert packed == 3 * (MiB // 2 + MiB // 64) + 2048 + 64
    need = sum(1 for r in range(n) for l in range(L) if r not in _owners(cfg, l))
    assert _core.sim_fabric_bytes(key) == need * packed  # every remote copy moved packed
    assert res[0].engine_stats["verify_failures"] == 0


@pytest.mark.parametrize("mode,policy", [(1, {}), (2, {}), (3, {}), (0, {"relay": True}), (0, {"collective": True})])
def test_fp8_store_bf16_fused_unpack_on_landing(mode, policy):
    """--store bf16: every chunk that becomes resident - received, relayed,
    broadcast (mode 0 ncclBroadcast) or staged - goes through the fused
    verify+unpack (CRC of the packed chunk and its bf16 image in one pass), so
    every rank ends with the same dequantized layer."""
    n, L, size = 4, 6, 3 * MiB + 4096
    cfg = make_workload(n, L, size, tier="host", seeding="leader" if mode == 0 else "random", chunk_bytes=MiB)

    def check(rts):
        for l in range(L):
            packed = _core.fp8_pack_layer_host(_core.fill_random_host(size, layer_seed(0, l)), MiB, 128)
            want = _core.fp8_unpack_layer_host(packed, size, MiB, 128)
            for r in rts:
                assert r.unpacked_layer_bytes(l) == want, (r.node_id, l)

    (res,), _ = run_cluster(cfg, mode, rt_kw={"pack": "fp8", "store": "bf16"}, inspect=check, pull_window=n - 1,
                            **policy)
    assert all(r.engine_stats["verify_failures"] == 0 and r.engine_stats["unverified_pieces"] == 0 for r in res)


@pytest.mark.parametrize("store", ["packed", "bf16"])
def test_relays_around_slow_link_cut_on_chunk_grid(store):
    """Mode 1 "links" policy with a slow link in the plan and layers whose size
    is not a grid multiple: the relay slices moved off the slow link end on
    chunk boundaries (the odd tail chunk moves whole), so no chunk arrives as
    two partial pieces from different senders - every received chunk is
    CRC-checked (and with --store bf16 dequantized)."""
    n, L = 4, 4
    pack = store == "bf16"
    size = 4 * MiB + (512 if pack else 13)
    cfg = make_workload(n, L, size, tier="host", seeding="random", chunk_bytes=MiB)
    fast, slow = int(50e9), int(5e9)
    link_bw = {(a, b): fast for a in range(n) for b in range(n) if a != b}
    link_bw[(0, 1)] = link_bw[(1, 0)] = slow
    kw = {"pack": "fp8", "store": "bf16"} if pack else {}
    (res,), _ = run_cluster(cfg, 1, rt_kw=kw, owner_policy="links", link_bw=link_bw)
    for r in res:
        assert r.engine_stats["verify_failures"] == 0
        assert r.engine_stats["unverified_pieces"] == 0, r.engine_stats


def _owners(cfg, layer):
    return {nd.id for nd in cfg.nodes for per in nd.initial_layers.values() if layer in per}


def test_fp8_rejects_layer_sizes_off_the_scale_block():
    """fp8 packs whole bf16 scale blocks: a layer size that is not a multiple of
    2 x block bytes is refused up front with a clear error (not a kernel error)."""
    cfg = make_workload(1, 2, 2 * MiB + 13, tier="host", chunk_bytes=MiB)
    with pytest.raises(ValueError, match="multiples of 256 B"):
        Runtime(cfg, 0, engine="sim", registry={0: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=f"sim{next(_keys)}",
                pack="fp8")


def test_fp8_unpacked_layer_roundtrip_disk(tmp_path):
    cfg = make_workload(3, 4, 2 * MiB, tier="disk", seeding="random", chunk_bytes=MiB)
    key = f"sim{next(_keys)}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key,
                   storage_path=str(tmp_path), pack="fp8") for i in range(3)]
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
        for r in rts:
            for l in range(4):
                src = _core.fill_random_host(2 * MiB, layer_seed(0, l))
                packed = _core.fp8_pack_layer_host(src, MiB, 128)
                assert r.layer_bytes(l) == packed
                assert r.unpacked_layer_bytes(l) == _core.fp8_unpack_layer_host(packed, 2 * MiB, MiB, 128)
    finally:
        for r in rts:
            r.close()


# ------------------------------------------------------------- fault injection / NACK


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_corrupted_chunks_are_nacked_and_resent(mode):
    """--inject drop-chunk=P: received chunks are damaged behind their P2P group;
    the CRC check catches each one, the receiver NACKs it, the leader re-sends
    it from a pre-session holder, and the session still delivers exact bytes."""
    n = 4
    seeding = "leader" if mode == 0 else "random"
    cfg = make_workload(n, 6, 3 * MiB, tier="host", seeding=seeding, chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, mode, rt_kw={"inject_corrupt": 0.25, "inject_seed": 7, "max_retries": 8},
                              pull_window=2)
    injected = sum(r.engine_stats["injected"] for r in res)
    assert injected > 0
    failures = sum(r.engine_stats["verify_failures"] for r in res)
    # A damaged chunk may already have been forwarded (relays cut through before
    # the check), so its downstream receivers detect and NACK it as well.
    assert failures >= injected
    assert res[0].nacks == failures


def test_corruption_beyond_retry_budget_fails_loudly():
    cfg = make_workload(2, 1, 2 * MiB, tier="host", seeding="leader", chunk_bytes=MiB)
    key = f"sim{next(_keys)}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key,
                   inject_corrupt=1.0, max_retries=2) for i in range(2)]
    reg = {i: r.transport.address() for i, r in enumerate(rts)}
    for r in rts:
        r.transport.set_registry(reg)
    try:
        for r in rts:
            r.prepare(1)
        res = [None] * 2
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(4))) for i in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert not res[1].ok and "retries exhausted" in res[1].error
        assert not res[0].ok
    finally:
        for r in rts:
            r.close()


def test_client_held_layer_on_planned_engine():
    """C17 on the GPU data plane: node 1's external client holds layer 9. The
    leader plans node 1 as its sender; node 1's engine asks the client
    (ClientReq), stages the streamed bytes into its HBM slot, then forwards."""
    from distributed_llm_dissemination_amd.utils.config import ClientConf

    size = 2 * MiB + 4096
    cfg = make_workload(3, 3, size, tier="host", seeding="random", chunk_bytes=MiB)
    cfg.clients.append(ClientConf(id=1, addr="", layers={9: 0}))
    for r in range(3):
        cfg.assignment[r].append(9)
    key = f"sim{next(_keys)}"
    data = _core.fill_random_host(size, layer_seed(0, 9))
    ct = _core.tcp_transport("127.0.0.1:0", {}, True)
    client = _core.ClientNode(1, ct, {9: _core.LayerSrc.inmem(data, 0)})
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
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert all(x.ok for x in res), [x.error for x in res]
        for r in rts:
            assert r.layer_bytes(9) == data
            for l in range(3):
                assert r.layer_bytes(l) == _core.fill_random_host(size, layer_seed(0, l))
    finally:
        for r in rts:
            r.close()
        client.stop()
        ct.close()


@pytest.mark.parametrize("n", [4, 8])
@pytest.mark.parametrize("lanes", [1, -1, 0])
def test_mode1_balanced_seeding_forms_full_all_to_all_rounds(n, lanes):
    """The headline bench's schedule: with every rank seeding the same number of
    layers, each round moves one chunk to and one chunk from every peer
    (n - 1 sends + n - 1 recvs), so all xGMI links of every GPU are busy in
    every round. One lane: each round is one P2P group; world-1 lanes: one
    group per ring distance (a send and a recv); the default, one lane per
    directed link: one single-op group per link and direction."""
    layers, chunks = 2 * n, 4
    cfg = make_workload(n, layers, chunks * MiB, tier="host", seeding="random", chunk_bytes=MiB)
    (res,), _ = run_cluster(cfg, 1, rt_kw={"engine_opts": {"lanes": n - 1 if lanes == -1 else lanes}})
    per_rank_rounds = (layers // n) * chunks
    nl = {1: 1, -1: n - 1, 0: 2 * (n - 1)}[lanes]
    for r in res:
        assert r.engine_stats["groups"] == per_rank_rounds * nl
        assert r.engine_stats["pieces"] == per_rank_rounds * 2 * (n - 1)


def test_source_pool_shares_host_buffers():
    """--source-pool P: host-tier layers share P distinct pinned source buffers
    (layer l carries buffer l % P), so 126 x 3 GiB bf16 sources fit host memory;
    every layer is still delivered and CRC-verified from its own manifest."""
    n, L, size = 3, 7, 2 * MiB
    cfg = make_workload(n, L, size, tier="host", seeding="random", chunk_bytes=MiB)

    def check(rts):
        for r in rts:
            assert len(r._pool) <= 2
            for l in range(L):
                assert r.layer_bytes(l) == _core.fill_random_host(size, layer_seed(0, l, 2)), (r.node_id, l)

    (res,), _ = run_cluster(cfg, 1, rt_kw={"source_pool": 2}, inspect=check)
    assert res[0].engine_stats["verify_failures"] == 0


@pytest.mark.parametrize("n", [2, 4])
def test_disk_tier_more_chunks_than_the_bounce_ring(tmp_path, n):
    """Disk-tier layers of 12 chunks with an 8-buffer bounce ring (config #4
    shape at N > 1). A bounce buffer returns to the ring when its H2D copy has
    landed; held until the chunk's CRC check instead, the in-order verify queue
    (checks behind recvs that wait on the peer, whose sends wait on disk reads
    of its own) held every buffer on both ranks - a deadlock."""
    cfg = make_workload(n, 2 * n, 12 * MiB, tier="disk", seeding="random", chunk_bytes=MiB)
    (res,), _ = run_cluster(cfg, 1, rt_kw={"storage_path": str(tmp_path)})
    assert all(r.engine_stats["verify_failures"] == 0 for r in res)


@pytest.mark.parametrize("n", [3, 8])
@pytest.mark.parametrize("pack", ["none", "fp8"])
def test_mode0_host_share_stages_a_slice_per_rank(n, pack):
    """BASELINE config #2 from host memory with --host-share: the leader's host
    layers live in node-shared memory every rank maps, so each rank stages one
    slice per layer over its own host link and sends it to every other dest.
    Bytes arrive exact and verified (the leader's job CRCs check the slices its
    peers stage), and the leader's own link carries 1/n of the bytes instead
    of everything."""
    import threading as th

    L, size = 4, 8 * MiB
    cfg = make_workload(n, L, size, tier="host", seeding="leader", chunk_bytes=MiB)
    key = f"hs{next(_keys)}"
    rts = [None] * n

    def make(i):
        rts[i] = Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key,
                         host_share=True, pack=pack)

    ths = [th.Thread(target=make, args=(i,)) for i in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    try:
        assert all(r is not None for r in rts)
        assert all(sorted(r.shared_mapped) == list(range(L)) for r in rts[1:])
        reg = {i: r.transport.address() for i, r in enumerate(rts)}
        for r in rts:
            r.transport.set_registry(reg)
            r.unlink_shared()
        for r in rts:
            r.prepare(0)
        res = [None] * n
        go = [th.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(30))) for i in range(n)]
        for t in go:
            t.start()
        for t in go:
            t.join()
        assert all(x.ok for x in res), [x.error for x in res]
        for i, r in enumerate(rts):
            for l in cfg.assignment.get(i, []):
                assert r.layer_bytes(l) == expected_image(r, l, size), (i, l)
            st = r.engine.stats()
            assert st.verify_failures == 0 and st.unverified_pieces == 0
        slot = rts[0].slot_sizes[0]
        # every rank staged about 1/n of the bytes; the leader sent its slice to each receiver
        staged = [r.engine.stats().bytes_staged for r in rts]
        assert staged[0] <= L * size // n + L * 2 * MiB, staged
        assert sum(rts[0].link_bytes()["sent"].values()) <= (n - 1) * L * (slot // n + slot // 8 + 1)
    finally:
        for r in rts:
            if r is not None:
                r.close()


def test_mode0_host_share_layers_with_fewer_chunks_than_ranks():
    """8 ranks, layers of 4 chunks: each layer is staged by 4 of the 8 ranks,
    the subset rotating from layer to layer so every rank stages about 1/8."""
    import threading as th

    n, L, size = 8, 8, 4 * MiB
    cfg = make_workload(n, L, size, tier="host", seeding="leader", chunk_bytes=MiB)
    key = f"hs{next(_keys)}"
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=MiB, sim_key=key, host_share=True)
           for i in range(n)]
    try:
        reg = {i: r.transport.address() for i, r in enumerate(rts)}
        for r in rts:
            r.transport.set_registry(reg)
        for r in rts:
            r.prepare(0)
        res = [None] * n
        go = [th.Thread(target=lambda i=i: res.__setitem__(i, rts[i].execute(30))) for i in range(n)]
        for t in go:
            t.start()
        for t in go:
            t.join()
        assert all(x.ok for x in res), [x.error for x in res]
        for i, r in enumerate(rts):
            for l in range(L):
                assert r.layer_bytes(l) == expected_image(r, l, size)
        staged = [r.engine.stats().bytes_staged for r in rts]
        assert staged == [L * size // n] * n, staged
    finally:
        for r in rts:
            r.close()


def test_mode2_planned_dest_loads_its_own_lower_tier_copy():
    """Mode 2 on the planned (GPU) engine: a dest that holds a layer in a lower
    tier (pinned host) loads it itself (min_loaded_sender); its one job is
    dispatched at once (window 1), so there is nothing pending for the peer to
    steal and the peer sends nothing of it."""
    cfg = make_workload(2, 2, 2 * MiB, tier="host", seeding="leader", chunk_bytes=MiB)
    cfg.assignment = {0: [0, 1], 1: [0]}
    cfg.nodes[1].initial_layers = {2: {0: 2 * MiB}}  # rank 1 holds layer 0 in host memory too

    def inspect(rts):
        assert rts[1].link_bytes()["recv"].get(0, 0) == 0  # nothing of layer 0 came from rank 0

    (res,), _ = run_cluster(cfg, 2, pull_window=1, inspect=inspect)
    assert res[1].engine_stats["bytes_staged"] == 2 * MiB


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_single_rank_verifies_every_staged_byte_once(mode):
    """One rank promoting 6 host-tier layers (the GPU engine test's workload,
    tests/test_gpu_engine.py): every staged byte is CRC-checked exactly once
    in every mode - the staging checks go out in batches of up to 16 chunks
    (PlannedEngine::flush_stage_checks) - session after session."""
    size = 6 * MiB + 4096
    cfg = make_workload(1, 6, size, tier="host", chunk_bytes=MiB)
    rt = Runtime(cfg, 0, engine="sim", chunk_bytes=MiB, registry={0: "127.0.0.1:0"}, sim_key=f"one{next(_keys)}")
    try:
        for _ in range(2):
            res = rt.run(mode, timeout=60)
            assert res.ok, res.error
            assert res.engine_stats["bytes_staged"] == 6 * size
            assert res.engine_stats["bytes_verified"] == 6 * size
            assert res.engine_stats["verify_failures"] == 0
            # 6 layers x 7 chunks, checked in batches of up to 16 per verify
            assert res.engine_stats["verify_chunks"] == 42
            assert res.engine_stats["verify_calls"] <= 42 // 4, res.engine_stats
            for l in range(6):
                assert rt.layer_bytes(l) == expected_image(rt, l, size)
    finally:
        rt.close()


def test_mode2_slow_self_load_is_stolen_by_a_faster_peer():
    """rank 1 holds layer 0 in a slow tier (LimitRate 4 MB/s) and
    must load it; rank 0 holds it in memory, unpaced. Rank 1 starts on its
    first range jobs itself (min_loaded_sender, its window of two own loads);
    rank 0, done with its own load, steals rank 1's pending ranges
    (node.go:1036-1042: the thief is at least as fast) and sends them. Byte
    counters: rank 1 staged the chunks of the ranges it started and received
    the others - most of the layer - from rank 0, every chunk once; every byte
    of the layer is checked at rank 1 (run_cluster)."""
    from distributed_llm_dissemination_amd.utils.config import SOURCE_MEM

    cfg = make_workload(2, 1, 8 * MiB, tier="host", seeding="leader", chunk_bytes=MiB)
    cfg.assignment = {0: [0], 1: [0]}
    cfg.nodes[1].initial_layers = {SOURCE_MEM: {0: 8 * MiB}}
    cfg.nodes[1].sources = {SOURCE_MEM: 4_000_000}

    (res,), _ = run_cluster(cfg, 2, pull_window=1, pull_job_bytes=MiB)
    staged, recv = res[1].engine_stats["bytes_staged"], res[1].engine_stats["bytes_recv"]
    assert staged >= MiB and recv >= 4 * MiB, res[1].engine_stats  # the slow tier was relieved
    assert staged + recv == 8 * MiB and res[1].engine_stats["scratch_landings"] == 0
    assert res[0].engine_stats["bytes_sent"] == recv
