"""Measure the node's NVMe read rate where the disk tier lives (bench.py --tier disk).

The disk tier reads layer files with O_DIRECT preads from several reader threads
per rank (PlannedEngine disk_readers), and at N > 1 every rank of a node reads
the same NVMe: the node-wide pacer and mode 3's disk group plan that one budget
(`node_disk_gbps`). A constant there is a guess about someone else's disk - on
the round-5 box the NVMe read 17.9-20 GB/s where the round-1 box read 13.3
(profiles/r5_disk/, profiles/r1_diskspeed.log) - so bench.py measures it once
per host before the run: write a probe file, fsync it (an O_DIRECT read of a
range with dirty pages would wait for their write-back), read it back with
O_DIRECT from `readers` threads, delete it. The C++ equivalent with the H2D leg
is bin/diskspeed.

Returns None where O_DIRECT is not available (tmpfs, some overlay mounts): the
caller keeps its default then.

``storage_info`` says what a directory sits on (file system type, device,
free bytes: /proc/mounts + statvfs), for the benchmark's JSON: a rate read
from tmpfs, or through a loop device whose backing file the host caches, is
not an NVMe rate.
"""

from __future__ import annotations

import mmap
import os
import threading
import time
from typing import Dict, Optional

_ALIGN = 4096
MEMORY_FS = {"tmpfs", "ramfs", "devtmpfs", "hugetlbfs"}


def read_mode(direct_bytes: int, buffered_bytes: int) -> str:
    """What a disk-tier session's reads were: "o_direct" (every byte past this
    OS's page cache), "buffered" (none), "mixed", or "none" (nothing read)."""
    if direct_bytes <= 0 and buffered_bytes <= 0:
        return "none"
    if buffered_bytes <= 0:
        return "o_direct"
    return "buffered" if direct_bytes <= 0 else "mixed"


def refusal(fs: str, mode: str, allow_buffered: bool) -> Optional[str]:
    """Why a disk-tier benchmark must not report its rate as a disk's (None: it may)."""
    if allow_buffered:
        return None
    if fs in MEMORY_FS:
        return f"the layer files sit on {fs} (memory), not a disk"
    if mode in ("buffered", "mixed"):
        return "layer files were read without O_DIRECT (the file system refused it): reads may come from memory"
    return None


def storage_info(directory: str) -> Dict[str, object]:
    """The mount holding `directory`: {"fs", "device", "mount", "avail_bytes"}
    (fs "?" when /proc/mounts is unreadable)."""
    os.makedirs(directory, exist_ok=True)
    path = os.path.realpath(directory)
    best = ("", "?", "?")
    try:
        with open("/proc/mounts") as f:
            for line in f:
                parts = line.split()
                if len(parts) < 3:
                    continue
                dev, mnt, fs = parts[0], parts[1].replace("\\040", " "), parts[2]
                if (path == mnt or path.startswith(mnt.rstrip("/") + "/")) and len(mnt) >= len(best[0]):
                    best = (mnt, dev, fs)
    except OSError:
        pass
    st = os.statvfs(path)
    out = {"fs": best[2], "device": best[1], "mount": best[0] or "?", "avail_bytes": st.f_bavail * st.f_frsize}
    if best[2] == "overlay" or best[1].startswith("/dev/loop"):
        # what O_DIRECT cannot promise here: the layer below is the host's
        out["note"] = ("container overlay / loop device: O_DIRECT bypasses this OS's page cache, but the store "
                       "below it belongs to the host and may serve reads from the host's memory")
    return out


def read_rate_gbps(directory: str, size_bytes: int = 1 << 30, block_bytes: int = 16 << 20,
                   readers: int = 4) -> Optional[float]:
    """O_DIRECT read rate (GB/s, 1e9 B/s) of a fresh `size_bytes` file in `directory`."""
    if not hasattr(os, "O_DIRECT"):
        return None
    block = max(_ALIGN, block_bytes // _ALIGN * _ALIGN)
    nblocks = max(1, size_bytes // block)
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f".diskprobe.{os.getpid()}")
    bufs = [mmap.mmap(-1, block) for _ in range(max(1, readers))]  # page-aligned, as O_DIRECT needs
    try:
        # bytes that do not compress or dedupe - different in every block: a
        # storage layer that did either would report a rate real layers never see
        import numpy as np

        rng = np.random.default_rng(int.from_bytes(os.urandom(8), "little"))
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        try:
            for i in range(nblocks):
                os.pwrite(fd, rng.bytes(block), i * block)
            os.fsync(fd)
            # the written pages must not serve the reads below from this OS's cache
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        finally:
            os.close(fd)
        try:
            fd = os.open(path, os.O_RDONLY | os.O_DIRECT)
        except OSError:
            return None
        try:
            nxt = [0]
            lock = threading.Lock()
            errors = []

            def reader(buf):
                view = memoryview(buf)
                while True:
                    with lock:
                        i = nxt[0]
                        nxt[0] += 1
                    if i >= nblocks:
                        return
                    try:
                        got = os.preadv(fd, [view], i * block)
                    except OSError as e:  # EINVAL: the file system refuses O_DIRECT
                        errors.append(e)
                        return
                    if got != block:
                        errors.append(OSError(f"short read {got} of {block}"))
                        return

            threads = [threading.Thread(target=reader, args=(b,)) for b in bufs]
            t0 = time.perf_counter()
            for t in threads:
                t.start()
            for t in threads:
                t.join()
            dt = time.perf_counter() - t0
        finally:
            os.close(fd)
        if errors or dt <= 0:
            return None
        return nblocks * block / dt / 1e9
    finally:
        for b in bufs:
            b.close()
        try:
            os.unlink(path)
        except OSError:
            pass
