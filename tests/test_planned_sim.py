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


def run_cluster(cfg, mode, sessions=1, chunk=MiB, **policy):
    key = f"sim{next(_keys)}"
    n = len(cfg.nodes)
    rts = [Runtime(cfg, i, engine="sim", registry={i: "127.0.0.1:0"}, chunk_bytes=chunk, sim_key=key) for i in range(n)]
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
                    assert r.layer_bytes(l) == _core.fill_random_host(sizes[l], layer_seed(0, l)), (i, l)
            out.append(res)
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


@pytest.mark.parametrize("n", [3, 8])
@pytest.mark.parametrize("relay", [True, False])
def test_mode0_broadcast_relay(n, relay):
    cfg = make_workload(n, 4, 4 * MiB, tier="host", seeding="leader", chunk_bytes=MiB)
    (res,), key = run_cluster(cfg, 0, relay=relay)
    moved = _core.sim_fabric_bytes(key)
    assert moved == (n - 1) * 4 * 4 * MiB  # relay moves the same bytes, spread over all links


def test_device_seeded_uneven_copies_mode1():
    cfg = make_workload(4, 12, 2 * MiB, tier="device", seeding="uniform", copies=2, seed=3, chunk_bytes=MiB)
    run_cluster(cfg, 1)


def test_pipeline_assignment_mode2_dynamic_batches():
    cfg = make_workload(4, 16, MiB + 512, tier="host", seeding="random", assignment="pipeline", chunk_bytes=MiB)
    run_cluster(cfg, 2, pull_window=1)


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
