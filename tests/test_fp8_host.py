"""Host reference of the fp8 wire format (csrc/core/fp8.cc) against torch fp32/fp64 references.

The format (core/fp8.h): per source chunk [e4m3fn codes][one f32 scale per block], the scale a
power of two 2^E with E the smallest integer >= -126 such that the block's finite amax <= 448 * 2^E.
The gfx950 kernels are checked against this host reference in test_gpu_kernels.py."""
import numpy as np
import torch

from distributed_llm_dissemination_amd import _core

from test_gpu_kernels import _fp8_reference, _scale_exp

MiB = 1 << 20


def _split(packed: bytes, src: int, chunk: int, block: int):
    pc = chunk // 2 + chunk // 2 // block * 4
    qs, ss = [], []
    for c, off in enumerate(range(0, src, chunk)):
        n = min(chunk, src - off) // 2
        base = np.frombuffer(packed, dtype=np.uint8, count=n + n // block * 4, offset=c * pc)
        qs.append(base[:n])
        ss.append(base[n:].view(np.float32))
    return torch.from_numpy(np.concatenate(qs)), torch.from_numpy(np.concatenate(ss))


def test_scale_exp_edges():
    a = torch.tensor([0.0, 448.0, 449.0, 224.0, 1.0, 1e-38, 3.3e38, 1e-4])
    assert _scale_exp(a).tolist() == [0, 0, 1, -1, -8, -126, 120, -22]


def test_host_pack_matches_torch_reference():
    torch.manual_seed(0)
    src, chunk, block = 2 * MiB + 4096, MiB, 128
    x = (torch.randn(src // 2) * torch.logspace(-4, 4, src // 2)).to(torch.bfloat16)
    x[5] = float("inf")
    x[700] = float("-inf")
    x[1000] = float("nan")
    packed = _core.fp8_pack_layer_host(x.view(torch.uint8).numpy().tobytes(), chunk, block)
    assert len(packed) == _core.fp8_packed_size(src, chunk, block)
    q, s = _split(packed, src, chunk, block)
    qr, sr = _fp8_reference(x, block)
    assert torch.equal(s, sr)
    assert bool((torch.frexp(s)[0] == 0.5).all())
    # the host converter is IEEE round-to-nearest-even, as torch's; NaN codes may differ in sign only
    nan = torch.isnan(x.float())
    assert torch.equal(q[~nan], qr[~nan])
    assert bool(((q[nan] & 0x7F) == 0x7F).all())


def test_host_unpack_is_exact_product():
    torch.manual_seed(1)
    src, chunk, block = 2 * MiB, MiB, 64
    x = (torch.randn(src // 2) * 37).to(torch.bfloat16)
    packed = _core.fp8_pack_layer_host(x.view(torch.uint8).numpy().tobytes(), chunk, block)
    out = _core.fp8_unpack_layer_host(packed, src, chunk, block)
    y = torch.from_numpy(np.frombuffer(out, dtype=np.uint8).copy()).view(torch.bfloat16)
    q, s = _split(packed, src, chunk, block)
    want = (q.view(torch.float8_e4m3fn).double().view(-1, block) * s.double()[:, None]).view(-1)
    # a power-of-two scale times an e4m3 value is exact in bf16 (3 mantissa bits < 8)
    assert torch.equal(y.double(), want)
    err = (y.float() - x.float()).abs()
    assert bool((err <= x.float().abs() * 2**-4 + s.repeat_interleave(block) * 2**-9).all())


def test_host_roundtrip_random_bit_patterns():
    """Random payload bytes as bf16 (NaN, +-inf, the top binade): NaN stays NaN, +-inf saturate,
    nothing finite unpacks to inf (blocks with E = 120 saturate their codes at 240)."""
    src, chunk, block = MiB, MiB, 128
    raw = _core.fill_random_host(src, 3)
    x = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).view(torch.bfloat16).float()
    packed = _core.fp8_pack_layer_host(raw, chunk, block)
    y = torch.from_numpy(np.frombuffer(_core.fp8_unpack_layer_host(packed, src, chunk, block),
                                       dtype=np.uint8).copy()).view(torch.bfloat16).float()
    _, s = _split(packed, src, chunk, block)
    assert bool((s == 2.0**120).any())  # the top binade is exercised
    assert torch.equal(torch.isnan(x), torch.isnan(y))
    fin = torch.isfinite(x)
    assert bool(torch.isfinite(y[fin]).all())
    err = (y - x).abs()
    assert bool(((err <= x.abs() * 0.0625 + s.repeat_interleave(block) * 2**-9) | ~fin).all())
    inf = torch.isinf(x)
    assert torch.equal(y[inf].sign(), x[inf].sign())
