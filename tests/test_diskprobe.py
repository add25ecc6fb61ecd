"""The O_DIRECT read-rate probe bench.py uses for the node's NVMe budget at N > 1, and the
disk tier's read-mode / file-system / page-cache reporting."""

import os

import pytest

from distributed_llm_dissemination_amd import _core
from distributed_llm_dissemination_amd.models.catalog import make_workload
from distributed_llm_dissemination_amd.parallel import simclock
from distributed_llm_dissemination_amd.parallel.runtime import Runtime
from distributed_llm_dissemination_amd.utils.diskprobe import read_mode, read_rate_gbps, refusal, storage_info

MiB = 1 << 20


def test_probe_measures_and_cleans_up(tmp_path):
    r = read_rate_gbps(str(tmp_path), size_bytes=32 << 20, block_bytes=4 << 20, readers=3)
    # None only where the file system refuses O_DIRECT; otherwise a real rate
    assert r is None or r > 0.0
    assert os.listdir(tmp_path) == []  # the probe file is gone


def test_probe_rounds_odd_sizes_to_whole_aligned_blocks(tmp_path):
    # a block size that is not a 4 KiB multiple and a size smaller than one block:
    # one aligned block is read, never a short or misaligned O_DIRECT request
    r = read_rate_gbps(str(tmp_path / "sub"), size_bytes=1000, block_bytes=5000, readers=2)
    assert r is None or r > 0.0
    assert os.listdir(tmp_path / "sub") == []


# ---- the disk tier's honesty (bench.py --tier disk): what the reads were, where
# the files sit, whether the page cache held them (reference: conf/exe.sh:17
# drops every cache before a run; transport.go:351-367 sends from the file)


def test_read_mode_and_refusal_rules():
    assert read_mode(10, 0) == "o_direct" and read_mode(0, 10) == "buffered"
    assert read_mode(5, 5) == "mixed" and read_mode(0, 0) == "none"
    assert refusal("ext4", "o_direct", False) is None
    assert "memory" in refusal("tmpfs", "o_direct", False)  # a tmpfs run is never a disk rate
    assert "O_DIRECT" in refusal("xfs", "buffered", False)
    assert "O_DIRECT" in refusal("xfs", "mixed", False)
    assert refusal("tmpfs", "buffered", True) is None  # --allow-buffered: reported, not refused


def test_storage_info_names_the_mount(tmp_path):
    st = storage_info(str(tmp_path))
    assert st["fs"] not in ("", None) and st["avail_bytes"] > 0 and str(tmp_path).startswith(st["mount"])
    if os.path.isdir("/dev/shm"):
        assert storage_info("/dev/shm")["fs"] == "tmpfs"


def test_file_cache_drop_evicts_written_pages(tmp_path):
    p = tmp_path / "f.layer"
    p.write_bytes(os.urandom(8 * MiB))
    assert _core.file_cache_resident(str(p)) > 0.5  # just written: in the page cache
    left = _core.file_cache_drop(str(p))
    assert 0.0 <= left <= 0.05, left
    assert _core.file_cache_drop(str(tmp_path / "missing")) == -1


@pytest.mark.parametrize("o_direct", [True, False])
def test_disk_tier_counts_direct_and_buffered_bytes(tmp_path, o_direct):
    """The engine counts every disk-tier byte as read with O_DIRECT or buffered
    (the fallback when the file system refuses O_DIRECT: those may come from
    memory); Runtime.drop_disk_cache leaves no layer page cached."""
    if o_direct and storage_info(str(tmp_path))["fs"] in ("tmpfs",):
        pytest.skip("tmp_path is tmpfs")
    cfg = make_workload(2, 4, MiB, tier="disk", seeding="random", chunk_bytes=MiB // 4)
    key = f"dtier{os.getpid()}{o_direct}"
    with simclock.virtual_clock():
        reg = {i: f"{key}/{i}" for i in range(2)}
        rts = [Runtime(cfg, i, engine="sim", transport="inproc", registry=reg, chunk_bytes=MiB // 4, sim_key=key,
                       storage_path=str(tmp_path), engine_opts={"disk_o_direct": o_direct}) for i in range(2)]
        try:
            assert sum(len(r.disk_paths) for r in rts) == 4  # every layer file written once, by its holder
            assert max(r.drop_disk_cache() for r in rts) <= 0.05
            for r in rts:
                r.prepare(1)
            res, _ = simclock.run_ranks([lambda r=r: r.execute(60) for r in rts])
            assert all(x.ok for x in res), [x.error for x in res]
            direct = sum(x.engine_stats["disk_direct_bytes"] for x in res)
            buffered = sum(x.engine_stats["disk_buffered_bytes"] for x in res)
            assert direct + buffered == 4 * MiB  # each layer read from its file once
            assert read_mode(direct, buffered) == ("o_direct" if o_direct else "buffered")
        finally:
            for r in rts:
                r.close()
