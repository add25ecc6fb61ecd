"""gfx950 kernels as PyTorch ops (see kernels.py)."""

from .kernels import (  # noqa: F401
    crc32c,
    crc32c_values,
    fill_random_,
    fp8_pack,
    fp8_pack_layer,
    fp8_packed_size,
    fp8_unpack,
    fp8_verify_unpack,
    fp8_verify_unpack_chunks,
)

__all__ = [
    "crc32c",
    "crc32c_values",
    "fill_random_",
    "fp8_pack",
    "fp8_pack_layer",
    "fp8_packed_size",
    "fp8_unpack",
    "fp8_verify_unpack",
    "fp8_verify_unpack_chunks",
]
