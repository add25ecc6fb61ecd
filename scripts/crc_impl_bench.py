#!/usr/bin/env python3
"""Throughput of the CRC32C segment kernel on one MI355X, against read probes.

The kernel (csrc/kernels/crc32c.hip): slice-by-4 byte tables on lane-contiguous
64-B pieces of coalesced loads, one 1024-thread workgroup per CU; capped grids
(max_blocks) put more segments on every wave. The variants it replaced (nibble
tables on strided words, rolling byte-addressed nibble tables, MFMA GF(2)
products, directly loaded pieces, 4 recurrences per lane) and their numbers are
in profiles/r2_crc_ab. Shapes: 1 GiB in 64 MiB chunks (bulk throughput) and one
64 MiB chunk (the per-landing verify of the data engine). Prints one JSON object.
"""

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from distributed_llm_dissemination_amd import _core  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3


def main():
    quick = "--quick" in sys.argv  # default grid only (counter passes)
    n, chunk = 1 << 30, 64 << 20
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    _core.fill_random(buf.data_ptr(), n, 3)
    res = torch.empty(n // chunk, dtype=torch.int32, device="cuda")
    ws = torch.empty(_core.crc32c_workspace_bytes(n, chunk), dtype=torch.uint8, device="cuda")
    host = buf.cpu().numpy().tobytes()
    want = [_core.crc32c(host[i:i + chunk]) for i in range(0, n, chunk)]
    out = {}
    variants = [("slice", 0), ("slice_cap128", 128), ("slice_cap512", 512), ("slice_cap1024", 1024)]
    if quick:
        variants = [("slice", 0)]
    for name, cap in variants:
        def bulk():
            _core.crc32c_chunks_async(buf.data_ptr(), n, chunk, res.data_ptr(), ws.data_ptr(), 0, cap)

        def one():
            _core.crc32c_chunks_async(buf.data_ptr(), chunk, chunk, res.data_ptr(), ws.data_ptr(), 0, cap)

        t = timed(bulk, 20)
        out[f"{name}_1GiB_GBps"] = round(n / t / 1e9, 1)
        out[f"{name}_one_64MiB_us"] = round(timed(one, 100) * 1e6, 1)
        # the capped launch that was timed agrees with the host CRC32C of every chunk
        res.fill_(0)
        bulk()
        torch.cuda.synchronize()
        got = [int(x) & 0xFFFFFFFF for x in res.cpu().tolist()]
        out[f"{name}_match"] = got == want
    # Read roofline of this box for the same buffer: a read-only XOR stream.
    outx = torch.empty(4096 * 4, dtype=torch.int32, device="cuda")
    for blocks in (1024, 2048, 4096):
        for depth in (4, 8):
            t = timed(lambda: _core.read_xor_async(buf.data_ptr(), n, outx.data_ptr(), blocks, depth, 0), 20)
            out[f"read_xor_b{blocks}_d{depth}_GBps"] = round(n / t / 1e9, 1)
    # The CRC kernels' load shape without the CRC math (16 KiB per wave, 1024-thread
    # workgroups): layout 0 = each lane loads its own 64-B piece, 1 = every load instruction reads
    # one whole KiB (the CRC kernel's loads, before its in-register transpose).
    outs = torch.empty(1024 * 1024, dtype=torch.int32, device="cuda")
    for blocks in (256, 512):
        for layout in (0, 1):
            for roll in (False, True):
                t = timed(lambda: _core.read_seg_async(buf.data_ptr(), n, outs.data_ptr(), blocks, layout, roll, 0), 20)
                out[f"read_seg_b{blocks}_l{layout}_r{int(roll)}_GBps"] = round(n / t / 1e9, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
