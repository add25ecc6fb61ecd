// CRC32C (Castagnoli, reflected polynomial 0x82F63B78) host helpers.
//
// The reference has no integrity check beyond TCP checksums. We
// checksum every landed chunk on the GPU (csrc/kernels/crc32c.hip). The GPU
// kernel splits a chunk across lanes and waves and recombines the partial CRCs
// with GF(2) polynomial arithmetic: shifting a raw CRC over L zero bytes is a
// multiplication by x^(8L) mod P. These host helpers produce the tables and
// shift constants the kernel uses, and are the reference implementation the
// tests compare the kernel against.
#pragma once

#include <cstddef>
#include <cstdint>

namespace dissem {

constexpr uint32_t kCrc32cPoly = 0x82F63B78u;

// a(x) * b(x) mod P in the reflected representation (x^0 = 0x80000000).
uint32_t crc32c_multmodp(uint32_t a, uint32_t b);
// x^(8 * nbytes) mod P.
uint32_t crc32c_xpow8n(uint64_t nbytes);
// Raw CRC register after feeding `nbytes` zero bytes starting from `crc_raw`.
inline uint32_t crc32c_shift(uint32_t crc_raw, uint64_t nbytes) {
  return crc_raw ? crc32c_multmodp(crc32c_xpow8n(nbytes), crc_raw) : 0;
}
// Raw CRC (register starts at `crc`, no pre/post inversion).
uint32_t crc32c_raw(const void* data, size_t n, uint32_t crc = 0);
// Standard CRC32C (init 0xFFFFFFFF, xorout 0xFFFFFFFF); `crc` continues a previous value.
uint32_t crc32c(const void* data, size_t n, uint32_t crc = 0);
// Term that turns a raw CRC of an L-byte message into the standard CRC32C.
inline uint32_t crc32c_init_term(uint64_t nbytes) { return crc32c_shift(0xFFFFFFFFu, nbytes) ^ 0xFFFFFFFFu; }
// Slice-by-16 tables: T[k][v] = raw CRC of byte v followed by k zero bytes (16 x 256 entries).
void crc32c_slice16_tables(uint32_t* T);
// Byte-sliced linear map for shifting a register over `nbytes` zeros (4 x 256 entries).
void crc32c_shift_tables(uint64_t nbytes, uint32_t* A);

}  // namespace dissem
