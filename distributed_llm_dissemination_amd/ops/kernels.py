"""PyTorch-facing wrappers of the gfx950 kernels (csrc/kernels/*.hip).

Every op takes and returns CUDA (HIP) tensors and runs on the caller's current
stream, so it composes with PyTorch work without extra synchronization. Shapes,
dtypes, alignment and sizes are checked on the host before any launch (a kernel
must never be handed a buffer smaller than its grid assumes).

    import torch
    from distributed_llm_dissemination_amd import ops
    x = torch.randn(1 << 24, dtype=torch.bfloat16, device="cuda")
    q, s = ops.fp8_pack(x)                    # OCP e4m3fn + one f32 scale per 128 values
    y = ops.fp8_unpack(q, s)                  # bf16 again
    crc = ops.crc32c(x.view(torch.uint8), 64 << 20)   # CRC32C per 64 MiB chunk

These are the kernels the data engine runs itself (staging-time fp8 packing,
per-chunk CRC verification of every landed chunk); here they are usable on
their own, e.g. to check or unpack a layer a rank received.
"""

from __future__ import annotations

from typing import List, Tuple

import torch

from .. import _core

__all__ = [
    "fill_random_",
    "crc32c",
    "crc32c_values",
    "fp8_pack",
    "fp8_unpack",
    "fp8_pack_layer",
    "fp8_verify_unpack",
    "fp8_verify_unpack_chunks",
    "fp8_packed_size",
]

_FP8_BLOCKS = (32, 64, 128, 256, 512)


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check_dev(t: torch.Tensor, name: str, dtype=None, align: int = 16) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if t.data_ptr() % align:
        raise ValueError(f"{name} must be {align}-byte aligned")


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def fill_random_(t: torch.Tensor, seed: int) -> torch.Tensor:
    """Fill `t` with counter-based random bytes (splitmix64 of (seed, 8-byte index));
    byte-identical to `_core.fill_random_host(nbytes, seed)`."""
    _check_dev(t, "t", align=1)
    _core.fill_random(t.data_ptr(), _nbytes(t), seed, _stream())
    return t


def crc32c(t: torch.Tensor, chunk_bytes: int = 0) -> torch.Tensor:
    """CRC32C (Castagnoli) of every `chunk_bytes` chunk of `t`'s bytes (whole
    tensor when 0), as an int32 GPU tensor holding the uint32 bit patterns. One
    chunk may have any length; several need a chunk size that is a multiple of
    16 (every chunk starts 16-B aligned)."""
    _check_dev(t, "t")
    n = _nbytes(t)
    chunk = min(chunk_bytes or n, n)
    if n <= 0:
        return torch.empty(0, dtype=torch.int32, device=t.device)
    if chunk < n and chunk % 16:
        raise ValueError("chunk_bytes must be a multiple of 16 when the tensor holds several chunks")
    nchunks = (n + chunk - 1) // chunk
    out = torch.empty(nchunks, dtype=torch.int32, device=t.device)
    # the fold words of the launch: zeroed (kernels.h: the kernel leaves them zeroed)
    ws = torch.zeros(_core.crc32c_workspace_bytes(n, chunk), dtype=torch.uint8, device=t.device)
    _core.crc32c_chunks_async(t.data_ptr(), n, chunk, out.data_ptr(), ws.data_ptr(), _stream())
    return out


def crc32c_values(crcs: torch.Tensor) -> List[int]:
    """The unsigned CRC values of a `crc32c()` result (synchronizes)."""
    return [v & 0xFFFFFFFF for v in crcs.tolist()]


def fp8_pack(x: torch.Tensor, block: int = 128) -> Tuple[torch.Tensor, torch.Tensor]:
    """bf16 -> OCP fp8 e4m3fn with one power-of-two f32 scale per `block` values
    (2^E, the smallest E >= -126 with the block's finite amax <= 448 * 2^E; core/fp8.h).
    Non-finite inputs: +-inf saturate to +-448*scale, NaN stays NaN.
    Returns (q: float8_e4m3fn [n], scales: float32 [n / block])."""
    _check_dev(x, "x", torch.bfloat16)
    if block not in _FP8_BLOCKS:
        raise ValueError(f"block must be one of {_FP8_BLOCKS}")
    n = x.numel()
    if n % block:
        raise ValueError(f"numel ({n}) must be a multiple of block ({block})")
    q = torch.empty(n, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.empty(n // block, dtype=torch.float32, device=x.device)
    _core.fp8_pack(x.data_ptr(), n, q.data_ptr(), s.data_ptr(), block, _stream())
    return q, s


def fp8_unpack(q: torch.Tensor, scales: torch.Tensor, block: int = 128) -> torch.Tensor:
    """Inverse of `fp8_pack`: bf16 values q * scale (round to nearest even)."""
    if q.dtype not in (torch.float8_e4m3fn, torch.uint8):
        raise ValueError("q must be float8_e4m3fn (or its uint8 bytes)")
    _check_dev(q, "q")
    _check_dev(scales, "scales", torch.float32, align=4)
    if block not in _FP8_BLOCKS:
        raise ValueError(f"block must be one of {_FP8_BLOCKS}")
    n = q.numel()
    if n % block or scales.numel() != n // block:
        raise ValueError("scales must hold one value per block of q")
    y = torch.empty(n, dtype=torch.bfloat16, device=q.device)
    _core.fp8_unpack(q.data_ptr(), scales.data_ptr(), n, y.data_ptr(), block, _stream())
    return y


def fp8_packed_size(src_bytes: int, chunk_bytes: int, block: int = 128) -> int:
    """Bytes of a bf16 layer of `src_bytes` in the chunked fp8 wire/HBM layout."""
    return _core.fp8_packed_size(src_bytes, chunk_bytes, block)


def fp8_pack_layer(x: torch.Tensor, chunk_bytes: int, block: int = 128) -> torch.Tensor:
    """A whole bf16 layer into the data engine's packed layout (core/fp8.h): per
    source chunk of `chunk_bytes`, [e4m3fn values][f32 scales]. Returns uint8."""
    _check_dev(x, "x", torch.bfloat16)
    src = _nbytes(x)
    if chunk_bytes <= 0 or chunk_bytes % 4096 or src % (2 * block):
        raise ValueError("chunk_bytes must be a positive multiple of 4096 and the layer a whole number of blocks")
    out = torch.empty(fp8_packed_size(src, chunk_bytes, block), dtype=torch.uint8, device=x.device)
    _core.fp8_pack_chunks(x.data_ptr(), src, chunk_bytes, block, out.data_ptr(), _stream())
    return out


def fp8_verify_unpack(packed: torch.Tensor, src_bytes: int, chunk_bytes: int,
                      block: int = 128) -> Tuple[torch.Tensor, torch.Tensor]:
    """One fused pass over a packed layer: CRC32C of every packed chunk and the
    dequantized bf16 layer. Returns (bf16 [src_bytes / 2], crcs int32 [chunks])."""
    _check_dev(packed, "packed", torch.uint8)
    if chunk_bytes <= 0 or chunk_bytes % 4096 or src_bytes % (2 * block) or block not in _FP8_BLOCKS:
        raise ValueError("bad chunk_bytes / src_bytes / block")
    pbytes = fp8_packed_size(src_bytes, chunk_bytes, block)
    if packed.numel() < pbytes:
        raise ValueError(f"packed holds {packed.numel()} bytes, the layout needs {pbytes}")
    pchunk = chunk_bytes // 2 + chunk_bytes // 2 // block * 4
    nchunks = (pbytes + pchunk - 1) // pchunk
    out = torch.empty(src_bytes // 2, dtype=torch.bfloat16, device=packed.device)
    crcs = torch.empty(nchunks, dtype=torch.int32, device=packed.device)
    ws = torch.zeros(_core.crc32c_workspace_bytes(pbytes, pchunk), dtype=torch.uint8, device=packed.device)
    _core.fp8_verify_unpack_async(packed.data_ptr(), src_bytes, chunk_bytes, block, out.data_ptr(), crcs.data_ptr(),
                                  ws.data_ptr(), _stream())
    return out, crcs


def fp8_verify_unpack_chunks(chunks: List[Tuple[torch.Tensor, int]], block: int = 128
                             ) -> Tuple[List[torch.Tensor], torch.Tensor]:
    """The engine's batched form: independent packed chunks [(packed uint8, src_len), ...]
    (each the core/fp8.h image of `src_len` bf16 bytes, up to `_core.crc32c_batch_max()`
    of them) checked and dequantized in ONE launch. Returns ([bf16 per chunk], crcs int32)."""
    if not chunks or len(chunks) > _core.crc32c_batch_max():
        raise ValueError(f"1 to {_core.crc32c_batch_max()} chunks per launch")
    if block not in _FP8_BLOCKS:
        raise ValueError(f"block must be one of {_FP8_BLOCKS}")
    outs, items = [], []
    dev = chunks[0][0].device
    for packed, src_len in chunks:
        _check_dev(packed, "packed", torch.uint8)
        if packed.device != dev:
            raise ValueError("every chunk of one launch must be on the same GPU")
        if src_len <= 0 or src_len % (2 * block):
            raise ValueError("src_len must be a positive multiple of 2 * block")
        need = src_len // 2 + src_len // 2 // block * 4
        if packed.numel() < need:
            raise ValueError(f"packed chunk holds {packed.numel()} bytes, its layout needs {need}")
        y = torch.empty(src_len // 2, dtype=torch.bfloat16, device=dev)
        outs.append(y)
        items.append((packed.data_ptr(), src_len, y.data_ptr()))
    crcs = torch.empty(len(chunks), dtype=torch.int32, device=dev)
    ws = torch.zeros(_core.crc32c_batch_workspace_bytes(), dtype=torch.uint8, device=dev)
    _core.fp8_verify_unpack_batch_async(items, block, crcs.data_ptr(), ws.data_ptr(), _stream())
    return outs, crcs
