"""The O_DIRECT read-rate probe bench.py uses for the node's NVMe budget at N > 1."""

import os

from distributed_llm_dissemination_amd.utils.diskprobe import read_rate_gbps


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
