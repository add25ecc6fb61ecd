#!/usr/bin/env python3
"""Kernel throughput on one MI355X: random fill, CRC32C verify, fp8 pack/unpack.

Each kernel runs on a buffer larger than the 256 MiB Infinity Cache so the
numbers are HBM-bound, timed with HIP events over several repetitions, and
reported as GB/s of bytes touched (read + write) against the ~6.3 TB/s measured
HBM copy ceiling.
"""

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from distributed_llm_dissemination_amd import _core  # noqa: E402


def timed(fn, reps=10):
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
    n = 1 << 30
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {}
    t = timed(lambda: _core.fill_random(buf.data_ptr(), n, 7))
    out["fill_random_GBps"] = n / t / 1e9
    chunk = 64 << 20
    nch = n // chunk
    # fold words of the verify launches: zeroed once (the kernels leave them zeroed)
    ws = torch.zeros(_core.crc32c_workspace_bytes(n, chunk), dtype=torch.uint8, device="cuda")
    res = torch.empty(nch, dtype=torch.int32, device="cuda")
    t = timed(lambda: _core.crc32c_chunks_async(buf.data_ptr(), n, chunk, res.data_ptr(), ws.data_ptr(), 0))
    out["crc32c_GBps"] = n / t / 1e9
    # the per-landing check sizes: scripts/verify_bench.py
    ne = n // 2
    x = buf.view(torch.bfloat16)[:ne]
    q = torch.empty(ne, dtype=torch.uint8, device="cuda")
    sc = torch.empty(ne // 128, dtype=torch.float32, device="cuda")
    y = torch.empty(ne, dtype=torch.bfloat16, device="cuda")
    t = timed(lambda: _core.fp8_pack(x.data_ptr(), ne, q.data_ptr(), sc.data_ptr(), 128))
    out["fp8_pack_GBps"] = (2 * ne + ne + ne // 32) / t / 1e9
    t = timed(lambda: _core.fp8_unpack(q.data_ptr(), sc.data_ptr(), ne, y.data_ptr(), 128))
    out["fp8_unpack_GBps"] = (ne + ne // 32 + 2 * ne) / t / 1e9
    # fp8 wire format: whole-layer pack into the chunked layout, and the fused
    # verify (CRC32C per packed chunk) + unpack (bf16) pass a consumer runs.
    src = n // 2  # 512 MiB of bf16
    pbytes = _core.fp8_packed_size(src, chunk, 128)
    packed = torch.empty(pbytes, dtype=torch.uint8, device="cuda")
    unpacked = torch.empty(src, dtype=torch.uint8, device="cuda")
    t = timed(lambda: _core.fp8_pack_chunks(buf.data_ptr(), src, chunk, 128, packed.data_ptr()))
    out["fp8_pack_chunks_GBps"] = (src + pbytes) / t / 1e9
    pchunk = chunk // 2 + chunk // 2 // 128 * 4
    ws2 = torch.zeros(_core.crc32c_workspace_bytes(pbytes, pchunk), dtype=torch.uint8, device="cuda")
    t = timed(lambda: _core.fp8_verify_unpack_async(packed.data_ptr(), src, chunk, 128, unpacked.data_ptr(),
                                                    res.data_ptr(), ws2.data_ptr(), 0))
    out["fp8_verify_unpack_GBps"] = (pbytes + src) / t / 1e9
    out["fp8_verify_unpack_ms_per_GiB_bf16"] = t * 1e3 * (1 << 30) / src
    t = timed(lambda: buf[: n // 2].copy_(buf[n // 2 :]))
    out["torch_copy_GBps"] = n / t / 1e9
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
