"""gfx950 kernel numerics vs host / PyTorch fp32 references."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev_bytes(n):
    return torch.empty(n, dtype=torch.uint8, device="cuda")


@pytest.mark.parametrize("n", [16, 1000, (1 << 20) + 7, 64 << 20])
def test_fill_random_matches_host(gpu, n):
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 99)
    torch.cuda.synchronize()
    assert t.cpu().numpy().tobytes() == gpu.fill_random_host(n, 99)


@pytest.mark.parametrize(
    "n,chunk",
    [
        (64 << 10, 64 << 10),
        ((1 << 20) + 16, 1 << 20),  # tail chunk of 16 bytes
        ((3 << 20) + 5, 1 << 20),  # byte tail (not a multiple of 16)
        (5 << 20, (1 << 20) + 4096),  # chunk not a multiple of the 64 KiB segment
        (7 << 20, 48 << 10),  # chunks smaller than a segment
        (64 << 20, 64 << 20),
        ((64 << 20) + (5 << 10) + 3, 64 << 20),  # short last chunk: its own segment shifts and init term
        (100 << 10, 100 << 10),  # a partial 16 KiB segment inside one chunk
        ((160 << 20) + 48, 64 << 20),  # bulk: every wave owns several segments (rolling prefetch)
    ],
)
def test_crc32c_chunks_match_host(gpu, n, chunk):
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 7 + n)
    torch.cuda.synchronize()
    host = t.cpu().numpy().tobytes()
    want = [gpu.crc32c(host[i : i + chunk]) for i in range(0, n, chunk)]
    assert gpu.crc32c_chunks(t.data_ptr(), n, chunk) == want


@pytest.mark.parametrize(
    "n,chunk",
    [
        ((3 << 20) + 5, 1 << 20),  # byte tail
        (5 << 20, (1 << 20) + 4096),  # partial segment at every chunk end
        (96 << 20, 64 << 20),  # short last chunk of whole segments
        ((520 << 20) + 4096, 64 << 20),  # several rounds of workgroups, last round in half segments
    ],
)
@pytest.mark.parametrize("cus", [0, 8, 32])
def test_crc32c_cus_and_workspace_reuse(gpu, n, chunk, cus):
    """The grid's last round is sized for the CUs the stream may use (a CU-masked
    verify stream passes its count), and the fold words in the workspace are
    left zeroed by every launch: the same workspace serves three launches."""
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 5 + n)
    torch.cuda.synchronize()
    host = t.cpu().numpy().tobytes()
    want = [gpu.crc32c(host[i : i + chunk]) for i in range(0, n, chunk)]
    nch = len(want)
    ws = torch.zeros(gpu.crc32c_workspace_bytes(n, chunk), dtype=torch.uint8, device="cuda")
    for rep in range(3):
        out = torch.zeros(nch, dtype=torch.int32, device="cuda")
        gpu.crc32c_chunks_async(t.data_ptr(), n, chunk, out.data_ptr(), ws.data_ptr(), 0, cus)
        torch.cuda.synchronize()
        assert [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()] == want, rep
        assert int(ws.count_nonzero()) == 0  # the launch left its fold words zeroed


@pytest.mark.parametrize(
    "n,chunk",
    [
        ((8 << 20) + 16, 16 << 10),  # 513 one-segment chunks: a range capped at the LDS fold slots
        (7 << 20, 48 << 10),  # 3-segment chunks
        ((2 << 20) + 48, 4 << 10),  # chunks shorter than a segment
    ],
)
@pytest.mark.parametrize("cus", [1, 2])
def test_crc32c_walk_ranges_spanning_many_chunks(gpu, n, chunk, cus):
    """The CRC-only walk gives each workgroup a contiguous range of segments and
    folds it per chunk in LDS slots: with one or two CUs a range would span
    hundreds of small chunks, so the host caps it at the slot count and
    launches more workgroups."""
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 77 + n)
    torch.cuda.synchronize()
    host = t.cpu().numpy().tobytes()
    want = [gpu.crc32c(host[i : i + chunk]) for i in range(0, n, chunk)]
    ws = torch.zeros(gpu.crc32c_workspace_bytes(n, chunk), dtype=torch.uint8, device="cuda")
    out = torch.zeros(len(want), dtype=torch.int32, device="cuda")
    gpu.crc32c_chunks_async(t.data_ptr(), n, chunk, out.data_ptr(), ws.data_ptr(), 0, cus)
    torch.cuda.synchronize()
    assert [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()] == want
    assert int(ws.count_nonzero()) == 0


def test_crc32c_batch_matches_host(gpu):
    # the chunks one P2P group lands: independent buffers of mixed sizes
    sizes = [64 << 20, (1 << 20) + 16, 100 << 10, 16, 48 << 10, 3 * (16 << 10) + 32]
    bufs = []
    for i, n in enumerate(sizes):
        t = _dev_bytes(n)
        gpu.fill_random(t.data_ptr(), n, 1000 + i)
        bufs.append(t)
    torch.cuda.synchronize()
    got = gpu.crc32c_batch([(t.data_ptr(), t.numel()) for t in bufs])
    assert got == [gpu.crc32c(t.cpu().numpy().tobytes()) for t in bufs]
    # the batched and per-buffer launches agree
    assert got == [gpu.crc32c_chunks(t.data_ptr(), t.numel(), t.numel())[0] for t in bufs]


@pytest.mark.parametrize("cus", [1, 7, 224])
def test_crc32c_batch_full_and_cus(gpu, cus):
    """A full batch (crc32c_batch_max items, the engine's staging batch) of mixed
    sizes, with the grid sized for few CUs (the masked verify stream) and the
    async form reusing one workspace."""
    nmax = gpu.crc32c_batch_max()
    sizes = [[64 << 20, 3 * (16 << 10) + 32, 16, (5 << 20) + 4096, 48 << 10][i % 5] for i in range(nmax)]
    bufs = []
    for i, n in enumerate(sizes):
        t = _dev_bytes(n)
        gpu.fill_random(t.data_ptr(), n, 2000 + i)
        bufs.append(t)
    torch.cuda.synchronize()
    want = [gpu.crc32c(t.cpu().numpy().tobytes()) for t in bufs]
    assert gpu.crc32c_batch([(t.data_ptr(), t.numel()) for t in bufs], 0, cus) == want
    ws = torch.zeros(gpu.crc32c_batch_workspace_bytes(), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        out = torch.zeros(nmax, dtype=torch.int32, device="cuda")
        gpu.crc32c_batch_async([(t.data_ptr(), t.numel()) for t in bufs], out.data_ptr(), ws.data_ptr(), 0, cus)
        torch.cuda.synchronize()
        assert [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()] == want


def test_crc32c_single_chunk_over_1gib(gpu):
    """One chunk larger than 1 GiB (a whole-tensor ops.crc32c of a big layer):
    its segments' shifts to the chunk end combine two segpow levels."""
    n = (1 << 30) + (3 << 20) + 4096 + 7
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 4242)
    torch.cuda.synchronize()
    want = gpu.crc32c(t.cpu().numpy().tobytes())
    assert gpu.crc32c_chunks(t.data_ptr(), n, n) == [want]
    assert gpu.crc32c_batch([(t.data_ptr(), n)]) == [want]


@pytest.mark.parametrize("n", [5, 16 + 7, (16 << 10) + 9, 59055800, (64 << 20) - 8])
def test_crc32c_single_chunk_any_length(gpu, n):
    """A layer whose size is not a multiple of 16 ends in such a chunk (the
    reference's experiment layers are 10,930,691,768 B: last 64 MiB-grid chunk
    59,055,800 B); the per-chunk check and the batched check take it."""
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 300 + n)
    torch.cuda.synchronize()
    want = gpu.crc32c(t.cpu().numpy().tobytes())
    assert gpu.crc32c_chunks(t.data_ptr(), n, n) == [want]
    assert gpu.crc32c_chunks(t.data_ptr(), n, 64 << 20) == [want]
    assert gpu.crc32c_batch([(t.data_ptr(), n), (t.data_ptr(), n - 1)]) == [
        want, gpu.crc32c(t.cpu().numpy().tobytes()[: n - 1])]


def test_crc32c_detects_single_bit_flip(gpu):
    n = 4 << 20
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 5)
    a = gpu.crc32c_chunks(t.data_ptr(), n, 1 << 20)
    t[3 * (1 << 20) + 12345] ^= 1
    b = gpu.crc32c_chunks(t.data_ptr(), n, 1 << 20)
    assert a[:3] == b[:3] and a[3] != b[3]


@pytest.mark.parametrize("cus", [2, 32, 0])
def test_crc32c_walk_runs_carry_exactly(gpu, cus):
    """With few CUs a wave walks a long run of one chunk's segments and carries
    its lanes' CRC states from segment to segment (crc_walk's walk_gap): the
    result matches the host, and a flipped bit in any block of a run's first,
    middle or last segment - or in a lane's first or last word - changes only
    its chunk."""
    n, chunk = (128 << 20) + (16 << 10) + 48, 64 << 20
    t = _dev_bytes(n)
    gpu.fill_random(t.data_ptr(), n, 31337)
    torch.cuda.synchronize()
    host = t.cpu().numpy().tobytes()
    want = [gpu.crc32c(host[i : i + chunk]) for i in range(0, n, chunk)]
    ws = torch.zeros(gpu.crc32c_workspace_bytes(n, chunk), dtype=torch.uint8, device="cuda")

    def crcs():
        out = torch.zeros(len(want), dtype=torch.int32, device="cuda")
        gpu.crc32c_chunks_async(t.data_ptr(), n, chunk, out.data_ptr(), ws.data_ptr(), 0, cus)
        torch.cuda.synchronize()
        return [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()]

    assert crcs() == want
    seg = 16 << 10
    for off in [0, 5 * seg + 3 * 4096 + 63, 1000 * seg + 64 * 37, chunk - 1, chunk + 17 * seg + 2 * 4096 + 4]:
        t[off] ^= 0x10
        got = crcs()
        t[off] ^= 0x10
        c = off // chunk
        assert got[c] != want[c] and got[:c] + got[c + 1 :] == want[:c] + want[c + 1 :], off


def _scale_exp(amax: torch.Tensor) -> torch.Tensor:
    """core/fp8.h scale: the smallest E >= -126 with amax <= 448 * 2^E (0 if amax == 0), exact in f64."""
    a = amax.double()
    _, k = torch.frexp(a)  # a = m * 2^k, m in [0.5, 1)
    e = k.long() - 10
    for _ in range(4):  # 448 * 2^(k - 10) < a always; the answer is k - 9 or k - 8
        e = torch.where(a > 448.0 * torch.pow(2.0, e.double()), e + 1, e)
    e = e.clamp(min=-126)
    return torch.where(a > 0, e, torch.zeros_like(e))


def _fp8_reference(x_bf16: torch.Tensor, block: int):
    """fp32 reference of the pack: per-block amax over finite values, scale 2^E (_scale_exp)."""
    x = x_bf16.float().view(-1, block)
    fin = torch.isfinite(x)
    amax = torch.where(fin, x.abs(), torch.zeros_like(x)).amax(dim=1)
    e = _scale_exp(amax)
    y = x * torch.pow(2.0, -e.double()).float()[:, None]
    hi = torch.where(e >= 120, 240.0, 448.0).float()[:, None]  # q * 2^120 must stay finite in bf16
    y = torch.where(torch.isnan(y), y, torch.maximum(torch.minimum(y, hi), -hi))
    q = y.to(torch.float8_e4m3fn)
    scale = torch.pow(2.0, e.double()).float()
    return q.view(torch.uint8).reshape(-1), scale


@pytest.mark.parametrize("block", [32, 128, 512])
def test_fp8_pack_matches_torch(gpu, block):
    n = 1 << 20
    x = (torch.randn(n, device="cuda") * 3).to(torch.bfloat16)
    q = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.empty(n // block, dtype=torch.float32, device="cuda")
    gpu.fp8_pack(x.data_ptr(), n, q.data_ptr(), s.data_ptr(), block)
    torch.cuda.synchronize()
    qr, sr = _fp8_reference(x.cpu(), block)
    torch.testing.assert_close(s.cpu(), sr, rtol=0, atol=0)
    qg = q.cpu()
    bad = (qg != qr).nonzero().flatten()
    # gfx950's v_cvt_pk_fp8_f32 double-rounds values within ~2^-20 of a rounding tie
    # (e.g. 168.0000153 -> 160 instead of 176): the code may then be the other
    # neighbor. Everything else must match IEEE round-to-nearest-even exactly.
    xf = x.float().cpu().view(-1, block)
    y = (xf / sr[:, None]).flatten()
    dec = lambda c: c.view(torch.float8_e4m3fn).float()  # noqa: E731
    for i in bad.tolist():
        a, b = dec(qg[i : i + 1]).item(), dec(qr[i : i + 1]).item()
        tie = 0.5 * (a + b)
        assert abs(int(qg[i]) - int(qr[i])) == 1, (float(y[i]), int(qg[i]), int(qr[i]))
        assert abs(float(y[i]) - tie) <= abs(tie) * 2**-18, (float(y[i]), a, b)
    assert len(bad) < n * 0.002


def test_fp8_roundtrip_random_bit_patterns(gpu):
    # Random payload bytes reinterpreted as bf16 include NaN/Inf: NaN stays NaN, +-inf saturate.
    n = 1 << 20
    raw = _dev_bytes(2 * n)
    gpu.fill_random(raw.data_ptr(), 2 * n, 3)
    x = raw.view(torch.bfloat16)
    q = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.empty(n // 128, dtype=torch.float32, device="cuda")
    y = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    gpu.fp8_pack(x.data_ptr(), n, q.data_ptr(), s.data_ptr(), 128)
    gpu.fp8_unpack(q.data_ptr(), s.data_ptr(), n, y.data_ptr(), 128)
    torch.cuda.synchronize()
    xf, yf = x.float().cpu(), y.float().cpu()
    assert torch.equal(torch.isnan(xf), torch.isnan(yf))
    fin = torch.isfinite(xf)
    assert bool(torch.isfinite(yf[fin]).all())  # top-binade blocks saturate at 240 (core/fp8.h sat_limit)
    blk_amax = torch.where(fin, xf.abs(), torch.zeros_like(xf)).view(-1, 128).amax(1)
    tol = (blk_amax / 448.0 * 0.07 + 1e-30).repeat_interleave(128)  # e4m3: 3 mantissa bits + bf16 rounding
    err = (yf - xf).abs()
    ok = (err <= tol + xf.abs() * 0.0625) | ~fin
    assert ok.all()
    inf = torch.isinf(xf)
    assert torch.equal(yf[inf].sign(), xf[inf].sign())


def _host_fp8_codes_close(got: bytes, want: bytes, n_q_per_chunk, pchunk):
    """q codes may differ by one near rounding ties (gfx950 double rounding); scales must match."""
    g = np.frombuffer(got, dtype=np.uint8)
    w = np.frombuffer(want, dtype=np.uint8)
    assert g.shape == w.shape
    diff = np.nonzero(g != w)[0]
    in_q = (diff % pchunk) < n_q_per_chunk(diff // pchunk)
    assert in_q.all(), "scale bytes differ"
    assert (np.abs(g[diff].astype(int) - w[diff].astype(int)) == 1).all()
    assert len(diff) < g.size * 0.002


@pytest.mark.parametrize("size,chunk,block", [(3 * (1 << 20) + 4096, 1 << 20, 128), (2 << 20, 1 << 20, 32),
                                              ((1 << 20) + 1024, 64 << 10, 512)])
def test_fp8_pack_chunks_matches_host_layout(gpu, size, chunk, block):
    x = (torch.randn(size // 2, device="cuda") * 2).to(torch.bfloat16)
    packed_n = gpu.fp8_packed_size(size, chunk, block)
    out = _dev_bytes(packed_n)
    gpu.fp8_pack_chunks(x.data_ptr(), size, chunk, block, out.data_ptr())
    torch.cuda.synchronize()
    want = gpu.fp8_pack_layer_host(x.view(torch.uint8).cpu().numpy().tobytes(), chunk, block)
    pchunk = chunk // 2 + chunk // 2 // block * 4
    last_q = (size % chunk) // 2 if size % chunk else chunk // 2

    def n_q(c):
        return np.where(c == (packed_n - 1) // pchunk, last_q, chunk // 2)

    _host_fp8_codes_close(out.cpu().numpy().tobytes(), want, n_q, pchunk)


def _torch_unpack(packed: torch.Tensor, src_len: int, block: int) -> torch.Tensor:
    """fp32 PyTorch reference of one packed chunk's dequantization: e4m3fn -> f32,
    times its block's f32 scale, rounded to bf16 (core/fp8.h layout [q][scales])."""
    n = src_len // 2
    q = packed[:n].view(torch.float8_e4m3fn).float()
    sc = packed[n : n + n // block * 4].view(torch.float32)
    return (q.view(-1, block) * sc[:, None]).view(-1).to(torch.bfloat16)


def _assert_bf16_bits_equal(got: torch.Tensor, want: torch.Tensor):
    """Bit for bit, except that any NaN matches any NaN (payloads may differ)."""
    g, w = got.view(torch.bfloat16), want.view(torch.bfloat16)
    gn, wn = torch.isnan(g), torch.isnan(w)
    assert torch.equal(gn, wn)
    assert torch.equal(g.view(torch.int16)[~gn], w.view(torch.int16)[~wn])


@pytest.mark.parametrize("block", [32, 128, 512])
def test_fp8_unpack_matches_torch_fp32(gpu, block):
    """The standalone unpack kernel against the fp32 torch reference, on random
    bit patterns packed by the kernel (NaN codes and every scale exponent)."""
    size, chunk = 4 << 20, 4 << 20
    raw = _dev_bytes(size)
    gpu.fill_random(raw.data_ptr(), size, 31 + block)
    packed = _dev_bytes(gpu.fp8_packed_size(size, chunk, block))
    gpu.fp8_pack_chunks(raw.data_ptr(), size, chunk, block, packed.data_ptr())
    n = size // 2
    y = _dev_bytes(size)
    gpu.fp8_unpack(packed.data_ptr(), packed.data_ptr() + n, n, y.data_ptr(), block)
    torch.cuda.synchronize()
    _assert_bf16_bits_equal(y.view(torch.bfloat16), _torch_unpack(packed, size, block))


@pytest.mark.parametrize("size,chunk,block,cus", [
    (3 * (1 << 20) + 4096, 1 << 20, 128, 0), (2 << 20, 1 << 20, 64, 0), ((1 << 20) + 1024, 64 << 10, 512, 0),
    (64 << 20, 64 << 20, 128, 0), (2 << 20, 1 << 20, 256, 0), (2 << 20, 1 << 20, 32, 0),
    # more workgroups than slots with a short last round -> that round in half
    # segments (short segments inside it); the small sizes above run every segment in halves
    (160 << 20, (5 << 20) + 4096, 128, 0), (512 << 20, 64 << 20, 128, 0),
    # grids sized for few CUs (a masked verify stream): other split points
    (48 << 20, 16 << 20, 128, 3), ((24 << 20) + 4096, 1 << 20, 256, 7), (16 << 20, (1 << 20) + 4096, 64, 1),
    (8 << 20, 4 << 20, 32, 2), ((8 << 20) + 1024, 64 << 10, 512, 5), (136 << 20, 64 << 20, 128, 128)])
def test_fp8_fused_verify_unpack(gpu, size, chunk, block, cus):
    """One pass: CRC32C of every packed chunk + bf16 dequantization; compared with
    the CRC kernel, the host CRC, the fp32 torch reference of the unpack, the
    standalone unpack kernel and the host C++ unpack."""
    raw = _dev_bytes(size)
    gpu.fill_random(raw.data_ptr(), size, 11)  # random bf16 bit patterns, NaN/Inf included
    packed_n = gpu.fp8_packed_size(size, chunk, block)
    packed = _dev_bytes(packed_n)
    gpu.fp8_pack_chunks(raw.data_ptr(), size, chunk, block, packed.data_ptr())
    out = _dev_bytes(size)
    crcs = gpu.fp8_verify_unpack(packed.data_ptr(), size, chunk, block, out.data_ptr(), cus=cus)
    pchunk = chunk // 2 + chunk // 2 // block * 4
    assert crcs == gpu.crc32c_chunks(packed.data_ptr(), packed_n, pchunk)
    host = packed.cpu().numpy().tobytes()
    assert crcs == [gpu.crc32c(host[o : o + pchunk]) for o in range(0, packed_n, pchunk)]
    ref = _dev_bytes(size)
    for c, off in enumerate(range(0, size, chunk)):
        n = min(chunk, size - off) // 2
        base = packed.data_ptr() + c * pchunk
        gpu.fp8_unpack(base, base + n, n, ref.data_ptr() + off, block)
        _assert_bf16_bits_equal(out[off : off + 2 * n].view(torch.bfloat16),
                                _torch_unpack(packed[c * pchunk : c * pchunk + pchunk], 2 * n, block))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert out.cpu().numpy().tobytes() == gpu.fp8_unpack_layer_host(host, size, chunk, block)


@pytest.mark.parametrize("block,cus", [(128, 0), (128, 128), (32, 0), (512, 32), (64, 1)])
def test_fp8_fused_batch(gpu, block, cus):
    """The engine's launch: up to crc32c_batch_max independent packed chunks of
    mixed sizes (full 64 MiB grid chunks, a layer's short last chunk, chunks
    below one 16 KiB segment) in one launch; every CRC equals the host CRC of
    its packed bytes and every bf16 output the fp32 torch reference. The same
    workspace serves two launches (the kernel leaves its fold words zeroed)."""
    nmax = gpu.crc32c_batch_max()
    lens = [[64 << 20, (3 << 20) + 8 * block, 4 * block, (16 << 10) + 2 * block, 1 << 20][i % 5] for i in range(nmax)]
    lens = [n - n % (2 * block) for n in lens]
    chunks = []
    for i, n in enumerate(lens):
        raw = _dev_bytes(n)
        gpu.fill_random(raw.data_ptr(), n, 500 + i)
        p = _dev_bytes(gpu.fp8_packed_size(n, n, block))
        gpu.fp8_pack_chunks(raw.data_ptr(), n, n, block, p.data_ptr())
        chunks.append((p, n))
    ws = torch.zeros(gpu.crc32c_batch_workspace_bytes(), dtype=torch.uint8, device="cuda")
    for rep in range(2):
        outs = [_dev_bytes(n) for _, n in chunks]
        crc = torch.zeros(nmax, dtype=torch.int32, device="cuda")
        gpu.fp8_verify_unpack_batch_async([(p.data_ptr(), n, o.data_ptr()) for (p, n), o in zip(chunks, outs)],
                                          block, crc.data_ptr(), ws.data_ptr(), 0, cus)
        torch.cuda.synchronize()
        got = [int(x) & 0xFFFFFFFF for x in crc.cpu().tolist()]
        assert got == [gpu.crc32c(p.cpu().numpy().tobytes()) for p, _ in chunks], rep
        for (p, n), o in zip(chunks, outs):
            _assert_bf16_bits_equal(o.view(torch.bfloat16), _torch_unpack(p, n, block))
    # the synchronous binding agrees
    outs = [_dev_bytes(n) for _, n in chunks]
    assert gpu.fp8_verify_unpack_batch([(p.data_ptr(), n, o.data_ptr()) for (p, n), o in zip(chunks, outs)],
                                       block, 0, cus) == got


def test_fp8_fused_verify_unpack_detects_corruption(gpu):
    size, chunk = 4 << 20, 1 << 20
    raw = _dev_bytes(size)
    gpu.fill_random(raw.data_ptr(), size, 5)
    packed_n = gpu.fp8_packed_size(size, chunk, 128)
    packed = _dev_bytes(packed_n)
    gpu.fp8_pack_chunks(raw.data_ptr(), size, chunk, 128, packed.data_ptr())
    out = _dev_bytes(size)
    good = gpu.fp8_verify_unpack(packed.data_ptr(), size, chunk, 128, out.data_ptr())
    pchunk = chunk // 2 + chunk // 2 // 128 * 4
    packed[2 * pchunk + chunk // 2 + 3] ^= 0x10  # a scale byte of chunk 2
    bad = gpu.fp8_verify_unpack(packed.data_ptr(), size, chunk, 128, out.data_ptr())
    assert [i for i in range(4) if good[i] != bad[i]] == [2]


@pytest.mark.parametrize("n,chunk", [(8 << 20, 2 << 20), ((64 << 20) + 16, 16 << 20)])
def test_rccl_selftest_p2p_and_broadcast(gpu, n, chunk):
    # One-rank communicator: ncclSend/ncclRecv to self in groups and an
    # in-place ncclBroadcast, issued through the engine's Backend::group.
    src, p2p, bcast = gpu.rccl_selftest(0, n, chunk)
    assert len(src) == (n + chunk - 1) // chunk
    assert p2p == src
    assert bcast == src


def test_crc_table_upload_never_waits_for_other_streams(gpu):
    """Round-3 hang: the first CRC of a new chunk size uploaded its tables with
    a null-stream hipMemcpy, which waited for every blocking stream - the comm
    lanes' RCCL kernels included - in the middle of a session. A kernel that
    spins on a host flag holds a blocking stream (an RCCL kernel waiting on a
    peer); a CRC of a never-seen size on another stream must launch without
    waiting for it, and still be right."""
    n = (40 << 20) + 3 * 4096 + 48  # a size no other test checks: fresh fold tables
    ms, iters, crc = gpu.crc_launch_beside_blocked_stream(n)
    assert ms < 250, ms           # before the fix: until the spin ran out (~2 s)
    assert iters < 600000, iters  # released by the host, not by its bound
    assert crc == gpu.crc32c(gpu.fill_random_host(n, 7))
