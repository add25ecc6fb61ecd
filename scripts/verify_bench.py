#!/usr/bin/env python3
"""Receive-side verify kernels at the size the engine launches them (one MI355X).

The data engine checks every landed 64 MiB chunk: plain CRC32C (the headline),
or with --pack fp8 --store bf16 the fused CRC32C + dequantization of the packed
chunk (33 MiB in, 64 MiB of bf16 out). It batches the chunks one P2P group or
one staging pass landed into one launch (up to crc32c_batch_max), the fold
inside the kernel. This prints, per case, the device time per 64 MiB source
chunk and the bytes moved per second:

  crc_single / fused_single   one chunk per launch (round 4's engine)
  crc_batch_K / fused_batch_K K chunks per launch (K = 1, 4, 8, 16)
  crc_bulk_1GiB               one launch over 1 GiB cut in 64 MiB chunks

Every launch reads chunks that are not in the 256 MiB Infinity Cache (a pool of
distinct buffers, cycled), and every case is checked once against the host CRC
and the standalone unpack. Run it under rocprofv3 --kernel-trace --stats for the
per-kernel device times (the HIP-event numbers here include launch gaps).

    python scripts/verify_bench.py [--reps 40] [--pool 24] [--cus N] [--only-full-batch]

--only-full-batch runs just the full-batch launches of both kernels (and the
checks), so a rocprofv3 --pmc pass sees one launch shape per kernel.
"""

import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from distributed_llm_dissemination_amd import _core  # noqa: E402

CHUNK = 64 << 20
BLOCK = 128


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--pool", type=int, default=24, help="distinct 64 MiB chunks cycled through (>= 16)")
    ap.add_argument("--cus", type=int, default=0, help="CUs the launches size their grid for (0: all)")
    ap.add_argument("--only-full-batch", action="store_true", help="only the full-batch launches (counter runs)")
    args = ap.parse_args()
    full_only = args.only_full_batch
    pool = max(16, args.pool)
    nmax = _core.crc32c_batch_max()
    out = {"chunk_MiB": CHUNK >> 20, "pool_chunks": pool, "cus": args.cus}

    # ---- plain CRC32C of 64 MiB chunks
    bufs = [torch.empty(CHUNK, dtype=torch.uint8, device="cuda") for _ in range(pool)]
    for i, b in enumerate(bufs):
        _core.fill_random(b.data_ptr(), CHUNK, 100 + i)
    torch.cuda.synchronize()
    want = [_core.crc32c(b.cpu().numpy().tobytes()) for b in bufs[:nmax]]
    ws = torch.zeros(_core.crc32c_batch_workspace_bytes(), dtype=torch.uint8, device="cuda")
    res = torch.zeros(nmax, dtype=torch.int32, device="cuda")
    calls = [0]

    def crc_single():
        i = calls[0] % pool
        calls[0] += 1
        _core.crc32c_chunks_async(bufs[i].data_ptr(), CHUNK, CHUNK, res.data_ptr(), ws.data_ptr(), 0, args.cus)

    if not full_only:
        t = timed(crc_single, args.reps)
        out["crc_single_us_per_chunk"] = round(t * 1e6, 1)
        out["crc_single_GBps"] = round(CHUNK / t / 1e9, 1)
    for k in (1, 4, 8, 16):
        if k > nmax or (full_only and k != nmax):
            continue
        calls[0] = 0

        def crc_batch(k=k):
            base = (calls[0] * k) % pool
            calls[0] += 1
            items = [(bufs[(base + j) % pool].data_ptr(), CHUNK) for j in range(k)]
            _core.crc32c_batch_async(items, res.data_ptr(), ws.data_ptr(), 0, args.cus)

        t = timed(crc_batch, args.reps)
        out[f"crc_batch_{k}_us_per_chunk"] = round(t * 1e6 / k, 1)
        out[f"crc_batch_{k}_GBps"] = round(k * CHUNK / t / 1e9, 1)
    res.zero_()
    _core.crc32c_batch_async([(b.data_ptr(), CHUNK) for b in bufs[:nmax]], res.data_ptr(), ws.data_ptr(), 0, args.cus)
    torch.cuda.synchronize()
    out["crc_batch_matches_host"] = [x & 0xFFFFFFFF for x in res.cpu().tolist()] == want
    if not full_only:
        # a lone chunk's launch by size: the intercept is the launch's fixed
        # cost (dispatch, table fill, first loads, last wave, fold), the slope its rate
        for mib in (1, 4, 16, 64):
            calls[0] = 0

            def crc_lone(mib=mib):
                i = calls[0] % pool
                calls[0] += 1
                _core.crc32c_chunks_async(bufs[i].data_ptr(), mib << 20, mib << 20, res.data_ptr(), ws.data_ptr(), 0,
                                          args.cus)

            out[f"crc_lone_{mib}MiB_us"] = round(timed(crc_lone, args.reps) * 1e6, 1)
        big = torch.empty(16 * CHUNK, dtype=torch.uint8, device="cuda")
        _core.fill_random(big.data_ptr(), big.numel(), 5)
        wsb = torch.zeros(_core.crc32c_workspace_bytes(big.numel(), CHUNK), dtype=torch.uint8, device="cuda")
        t = timed(lambda: _core.crc32c_chunks_async(big.data_ptr(), big.numel(), CHUNK, res.data_ptr(),
                                                    wsb.data_ptr(), 0, args.cus), args.reps // 2)
        out["crc_bulk_1GiB_GBps"] = round(big.numel() / t / 1e9, 1)
        del big
    del bufs

    # ---- fused CRC32C + fp8 -> bf16 of packed 64 MiB source chunks
    src = torch.empty(CHUNK, dtype=torch.uint8, device="cuda")
    pchunk = _core.fp8_packed_size(CHUNK, CHUNK, BLOCK)
    packed, outs = [], []
    for i in range(pool):
        _core.fill_random(src.data_ptr(), CHUNK, 900 + i)  # random bf16 bit patterns
        p = torch.empty(pchunk, dtype=torch.uint8, device="cuda")
        _core.fp8_pack_chunks(src.data_ptr(), CHUNK, CHUNK, BLOCK, p.data_ptr())
        packed.append(p)
        outs.append(torch.empty(CHUNK, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    moved = pchunk + CHUNK  # bytes read + written per chunk
    calls[0] = 0

    def fused_single():
        i = calls[0] % pool
        calls[0] += 1
        _core.fp8_verify_unpack_async(packed[i].data_ptr(), CHUNK, CHUNK, BLOCK, outs[i].data_ptr(), res.data_ptr(),
                                      ws.data_ptr(), 0, args.cus)

    if not full_only:
        t = timed(fused_single, args.reps)
        out["fused_single_us_per_chunk"] = round(t * 1e6, 1)
        out["fused_single_GBps"] = round(moved / t / 1e9, 1)
    for k in (1, 4, 8, 16):
        if k > nmax or (full_only and k != nmax):
            continue
        calls[0] = 0

        def fused_batch(k=k):
            base = (calls[0] * k) % pool
            calls[0] += 1
            items = [(packed[(base + j) % pool].data_ptr(), CHUNK, outs[(base + j) % pool].data_ptr())
                     for j in range(k)]
            _core.fp8_verify_unpack_batch_async(items, BLOCK, res.data_ptr(), ws.data_ptr(), 0, args.cus)

        t = timed(fused_batch, args.reps)
        out[f"fused_batch_{k}_us_per_chunk"] = round(t * 1e6 / k, 1)
        out[f"fused_batch_{k}_GBps"] = round(k * moved / t / 1e9, 1)
    # correctness of the batched launch: CRCs vs host, bf16 vs the standalone unpack
    res.zero_()
    for o in outs[:nmax]:
        o.zero_()
    _core.fp8_verify_unpack_batch_async([(packed[j].data_ptr(), CHUNK, outs[j].data_ptr()) for j in range(nmax)],
                                        BLOCK, res.data_ptr(), ws.data_ptr(), 0, args.cus)
    torch.cuda.synchronize()
    out["fused_batch_crc_matches_host"] = [x & 0xFFFFFFFF for x in res.cpu().tolist()] == [
        _core.crc32c(p.cpu().numpy().tobytes()) for p in packed[:nmax]]
    ref = torch.empty(CHUNK, dtype=torch.uint8, device="cuda")
    ok = True
    n = CHUNK // 2
    for j in range(nmax):
        _core.fp8_unpack(packed[j].data_ptr(), packed[j].data_ptr() + n, n, ref.data_ptr(), BLOCK)
        ok = ok and torch.equal(ref, outs[j])
    out["fused_batch_bf16_matches_unpack"] = ok
    if full_only:
        print(json.dumps(out))
        return
    # references: the standalone unpack of one chunk, a torch copy of 64 MiB
    t = timed(lambda: _core.fp8_unpack(packed[0].data_ptr(), packed[0].data_ptr() + n, n, ref.data_ptr(), BLOCK),
              args.reps)
    out["plain_unpack_one_chunk_us"] = round(t * 1e6, 1)
    t = timed(lambda: ref.copy_(outs[1]), args.reps)
    out["torch_copy_64MiB_us"] = round(t * 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
