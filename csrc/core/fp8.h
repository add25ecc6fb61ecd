// fp8 wire/storage format of a layer (BASELINE config #5: 126 x 3 GiB
// Llama-3.1-405B-sized layers, which only fit one MI355X's 288 GB of HBM as
// fp8; the reference has no packing, it moves opaque bytes).
//
// A bf16 layer is cut on the source chunk grid (`src_chunk` bytes). Source
// chunk c of n bf16 elements packs into one packed chunk:
//     [ q: n bytes of OCP e4m3fn ][ scales: n/block f32 ]
// with one scale per `block` consecutive elements. The scale is a power of two,
// 2^E with E the smallest integer such that amax <= 448 * 2^E over the block's
// finite values (E = 0 if none, E >= -126): an E8M0-valued scale (stored as
// f32), so gfx950's scaled conversions (v_cvt_scalef32_pk_bf16_fp8, which
// apply only the scale's exponent) dequantize a pair of values in one
// instruction, and q * 2^E is exact in bf16 (sat_limit keeps it finite). Packed chunks are laid end to end, so the
// packed layer has its own uniform chunk grid of packed_chunk(src_chunk) bytes
// and every transfer, CRC and retry runs on that grid unchanged.
#pragma once

#include <cstdint>
#include <stdexcept>

namespace dissem {
namespace fp8 {

inline int64_t packed_len(int64_t src_bytes, int block) {  // one chunk
  const int64_t n = src_bytes / 2;
  return n + (n / block) * 4;
}
inline int64_t packed_chunk(int64_t src_chunk, int block) { return packed_len(src_chunk, block); }
inline void check(int64_t src_bytes, int64_t src_chunk, int block) {
  if (block != 32 && block != 64 && block != 128 && block != 256 && block != 512)
    throw std::runtime_error("fp8 block must be 32, 64, 128, 256 or 512");
  if (src_chunk % (2 * block)) throw std::runtime_error("fp8 source chunk must hold whole scale blocks");
  if (src_bytes % (2 * block))
    throw std::runtime_error("fp8 packing needs a layer size that is a multiple of 2*block bytes");
}
inline int64_t packed_size(int64_t src_bytes, int64_t src_chunk, int block) {
  const int64_t full = src_bytes / src_chunk, tail = src_bytes % src_chunk;
  return full * packed_chunk(src_chunk, block) + (tail ? packed_len(tail, block) : 0);
}
// Inverse of packed_size (throws if `packed` is not a packed layer size).
inline int64_t source_size(int64_t packed, int64_t src_chunk, int block) {
  const int64_t pc = packed_chunk(src_chunk, block);
  const int64_t full = packed / pc, tail = packed % pc;
  // tail = t/2 + t/(2*block)*4 = t*(block+4)/(2*block) for t a multiple of 2*block
  const int64_t t = tail * 2 * block / (block + 4);
  if (packed_len(t, block) != tail) throw std::runtime_error("size is not a packed fp8 layer size");
  return full * src_chunk + t;
}

// E of a block's scale 2^E from its finite amax (>= 0): exact integer logic on
// the f32 bits (448 = 1.75 * 2^8), identical in the gfx950 pack kernel.
inline int scale_exp(uint32_t amax_bits) {
  if (amax_bits == 0) return 0;
  const int ef = int(amax_bits >> 23);
  if (ef == 0) return -126;  // f32 subnormal amax: the lowest normal scale
  const int e = ef - 127 - 8 + ((amax_bits & 0x7FFFFFu) > 0x600000u ? 1 : 0);
  return e < -126 ? -126 : e;
}

// Largest code magnitude of a block with scale 2^E: 448, except 240 at E = 120
// (only blocks whose amax is within 2^-4 of bf16's max get there), where
// 256 * 2^120 would overflow bf16 on unpack (the bf16 maximum is 255 * 2^120).
inline float sat_limit(int e) { return e >= 120 ? 240.0f : 448.0f; }

// Host reference (bit-exact with the gfx950 kernel except where the hardware
// converter double-rounds values within 2^-18 of a rounding tie).
uint8_t f32_to_e4m3(float x);  // RNE, finite |x| <= 448 expected, NaN -> 0x7F|sign
float e4m3_to_f32(uint8_t q);
void pack_host(const uint16_t* bf16, int64_t n, uint8_t* q, float* scales, int block);
void unpack_host(const uint8_t* q, const float* scales, int64_t n, uint16_t* bf16, int block);
// Whole layer: src_bytes of bf16 -> packed_size(...) bytes in the chunked layout.
void pack_layer_host(const uint8_t* src, int64_t src_bytes, int64_t src_chunk, int block, uint8_t* dst);
void unpack_layer_host(const uint8_t* packed, int64_t src_bytes, int64_t src_chunk, int block, uint8_t* dst);

}  // namespace fp8
}  // namespace dissem
