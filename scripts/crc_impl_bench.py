#!/usr/bin/env python3
"""A/B of the CRC32C segment kernels on one MI355X.

impl 1 = bank-private nibble tables, one 16 KiB segment per wave (the
per-landing check), 2 = byte-addressed tables with a rolling prefetch of each
wave's next segment (bulk; capped grids: more segments per wave), 0 = auto.
(The MFMA GF(2)-product kernel, an 8-waves-per-SIMD variant and rolling on
nibble tables lost this A/B and were removed: profiles/r2_crc_ab.)
Shapes: 1 GiB in 64 MiB chunks (bulk throughput) and one 64 MiB chunk (the
per-landing verify of the data engine). Prints one JSON object.
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
    quick = "--quick" in sys.argv  # one variant per kernel (counter passes)
    n, chunk = 1 << 30, 64 << 20
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    _core.fill_random(buf.data_ptr(), n, 3)
    res = torch.empty(n // chunk, dtype=torch.int32, device="cuda")
    ws = torch.empty(_core.crc32c_workspace_bytes(n, chunk), dtype=torch.uint8, device="cuda")
    host = buf.cpu().numpy().tobytes()
    want = [_core.crc32c(host[i:i + chunk]) for i in range(0, n, chunk)]
    out = {}
    variants = [("nibble", 1, 0), ("roll2", 2, 0), ("roll2_cap128", 2, 128), ("roll2_cap512", 2, 512), ("auto", 0, 0)]
    if quick:
        variants = [("nibble", 1, 0), ("roll2", 2, 0)]
    for name, impl, cap in variants:
        def bulk():
            _core.crc32c_chunks_async(buf.data_ptr(), n, chunk, res.data_ptr(), ws.data_ptr(), 0, impl, cap)

        def one():
            _core.crc32c_chunks_async(buf.data_ptr(), chunk, chunk, res.data_ptr(), ws.data_ptr(), 0, impl, cap)

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
    print(json.dumps(out))


if __name__ == "__main__":
    main()
