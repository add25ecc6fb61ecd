"""The torch-facing kernel ops (distributed_llm_dissemination_amd.ops) against
plain PyTorch fp32 / host references."""

import pytest
import torch

from distributed_llm_dissemination_amd import _core, ops

pytestmark = pytest.mark.gpu


def test_fill_and_crc32c_match_host():
    t = torch.empty((5 << 20) + 48, dtype=torch.uint8, device="cuda")
    ops.fill_random_(t, 77)
    host = t.cpu().numpy().tobytes()
    assert host == _core.fill_random_host(t.numel(), 77)
    crcs = ops.crc32c_values(ops.crc32c(t, 1 << 20))
    assert crcs == [_core.crc32c(host[i : i + (1 << 20)]) for i in range(0, len(host), 1 << 20)]
    assert ops.crc32c_values(ops.crc32c(t)) == [_core.crc32c(host)]


@pytest.mark.parametrize("block", [32, 128, 512])
def test_fp8_pack_unpack_vs_torch_fp32(block):
    torch.manual_seed(block)
    x = (torch.randn(1 << 20, device="cuda") * torch.logspace(-3, 3, 1 << 20, device="cuda")).to(torch.bfloat16)
    q, s = ops.fp8_pack(x, block)
    assert q.dtype == torch.float8_e4m3fn and s.numel() == x.numel() // block
    # fp32 reference of the scale: the power of two 2^E with amax / 448 <= 2^E < 2 amax / 448
    amax = x.float().view(-1, block).abs().amax(dim=1)
    assert bool((s >= amax / 448.0).all()) and bool((s < 2 * amax / 448.0).all())
    assert bool((torch.frexp(s)[0] == 0.5).all())  # powers of two
    # dequantized values vs the input: within e4m3 precision (3 mantissa bits)
    deq = q.float().view(-1, block) * s[:, None]
    err = (deq - x.float().view(-1, block)).abs()
    assert bool((err <= x.float().view(-1, block).abs() * 2**-3 + s[:, None] * 2**-9).all())
    # unpack == torch's own e4m3fn -> f32 -> (x scale) -> bf16
    y = ops.fp8_unpack(q, s, block)
    torch.testing.assert_close(y, (q.float().view(-1, block) * s[:, None]).view(-1).to(torch.bfloat16), rtol=0, atol=0)


def test_fp8_layer_fused_verify_unpack():
    src = 3 * (4 << 20) + 8192  # 3 full chunks + a short one
    x = torch.randn(src // 2, device="cuda").to(torch.bfloat16)
    packed = ops.fp8_pack_layer(x, 4 << 20)
    assert packed.numel() == ops.fp8_packed_size(src, 4 << 20)
    y, crcs = ops.fp8_verify_unpack(packed, src, 4 << 20)
    pchunk = (4 << 20) // 2 + (4 << 20) // 2 // 128 * 4
    assert ops.crc32c_values(crcs) == ops.crc32c_values(ops.crc32c(packed, pchunk))
    # per-chunk unpack with the standalone kernel gives the same bf16 layer
    parts = []
    for c, off in enumerate(range(0, src, 4 << 20)):
        n = min(4 << 20, src - off) // 2
        base = packed[c * pchunk : c * pchunk + n + n // 128 * 4]
        q = base[:n].view(torch.float8_e4m3fn)
        s = base[n:].view(torch.float32)
        parts.append(ops.fp8_unpack(q, s))
    assert torch.equal(y, torch.cat(parts))


def test_fp8_verify_unpack_chunks_batch_vs_torch_fp32():
    """The engine's batched form through the op: independent packed chunks of
    mixed sizes (a full 64 MiB chunk, a layer's short tail, small ones) in one
    launch; CRCs against the op's plain CRC of each packed image, bf16 against
    torch's e4m3fn -> f32 x scale -> bf16 of the same bytes."""
    sizes = [64 << 20, (3 << 20) + 8192, 256, 1 << 20]
    chunks, refs = [], []
    for i, src in enumerate(sizes):
        torch.manual_seed(i)
        x = (torch.randn(src // 2, device="cuda") * (10.0 ** (i - 2))).to(torch.bfloat16)
        packed = ops.fp8_pack_layer(x, (src + 4095) // 4096 * 4096)  # one chunk: [q: src/2][scales f32]
        n = src // 2
        q, sc = packed[:n].view(torch.float8_e4m3fn), packed[n:].view(torch.float32)
        refs.append((q.float().view(-1, 128) * sc[:, None]).view(-1).to(torch.bfloat16))
        chunks.append((packed, src))
    outs, crcs = ops.fp8_verify_unpack_chunks(chunks)
    assert ops.crc32c_values(crcs) == [ops.crc32c_values(ops.crc32c(p))[0] for p, _ in chunks]
    for y, ref in zip(outs, refs):
        torch.testing.assert_close(y, ref, rtol=0, atol=0)
    with pytest.raises(ValueError):
        ops.fp8_verify_unpack_chunks([(chunks[0][0], 100)])  # not a whole number of scale blocks
    with pytest.raises(ValueError):
        ops.fp8_verify_unpack_chunks(chunks * 5)  # more than one launch holds


def test_ops_reject_bad_operands():
    x = torch.zeros(100, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        ops.fp8_pack(x, 128)  # not a whole number of blocks
    with pytest.raises(ValueError):
        ops.fp8_pack(x.float(), 4)
    with pytest.raises(ValueError):
        ops.crc32c(torch.zeros(64, dtype=torch.uint8), 16)  # host tensor
    with pytest.raises(ValueError):
        ops.crc32c(torch.zeros(64, dtype=torch.uint8, device="cuda"), 24)  # several chunks, not 16-B aligned
    # one chunk of any length is fine (a packed chunk's image: 128 q bytes + 8 of scales)
    odd = torch.zeros(136, dtype=torch.uint8, device="cuda")
    assert ops.crc32c_values(ops.crc32c(odd)) == [_core.crc32c(bytes(136))]
    with pytest.raises(ValueError):
        ops.fp8_verify_unpack(torch.zeros(16, dtype=torch.uint8, device="cuda"), 1 << 20, 1 << 20)
