#include "core/fp8.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace dissem {
namespace fp8 {

namespace {
inline float bf16_to_f32(uint16_t b) {
  uint32_t u = uint32_t(b) << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return uint16_t((u >> 16) | 0x40);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}
}  // namespace

uint8_t f32_to_e4m3(float x) {
  const uint8_t sign = std::signbit(x) ? 0x80 : 0x00;
  if (std::isnan(x)) return uint8_t(sign | 0x7F);
  float a = std::fabs(x);
  if (a >= 448.0f) return uint8_t(sign | 0x7E);
  if (a < 0.015625f) {  // below 2^-6: subnormal, step 2^-9
    int q = int(std::nearbyint(std::ldexp(a, 9)));
    return uint8_t(sign | q);  // q == 8 is exactly the smallest normal's code
  }
  int e;
  std::frexp(a, &e);  // a = f * 2^e, f in [0.5, 1)
  e -= 1;             // a = m * 2^e, m in [1, 2)
  const float m = std::ldexp(a, -e);
  int q = int(std::nearbyint((m - 1.0f) * 8.0f));
  if (q == 8) {
    q = 0;
    ++e;
  }
  int code = ((e + 7) << 3) | q;
  if (code > 0x7E) code = 0x7E;
  return uint8_t(sign | code);
}

float e4m3_to_f32(uint8_t q) {
  const float s = (q & 0x80) ? -1.0f : 1.0f;
  const int e = (q >> 3) & 15, m = q & 7;
  if (e == 15 && m == 7) return std::copysign(NAN, s);
  if (e == 0) return s * std::ldexp(float(m), -9);
  return s * std::ldexp(1.0f + float(m) / 8.0f, e - 7);
}

void pack_host(const uint16_t* in, int64_t n, uint8_t* q, float* scales, int block) {
  for (int64_t b = 0; b < n / block; ++b) {
    float amax = 0.f;
    for (int i = 0; i < block; ++i) {
      float x = bf16_to_f32(in[b * block + i]);
      if (std::isfinite(x)) amax = std::fmax(amax, std::fabs(x));
    }
    uint32_t ab;
    memcpy(&ab, &amax, 4);
    const int e = scale_exp(ab);
    const float inv = std::ldexp(1.0f, -e);  // exact: x * 2^-E only moves the exponent
    const float hi = sat_limit(e);
    for (int i = 0; i < block; ++i) {
      float y = bf16_to_f32(in[b * block + i]) * inv;
      if (y == y) y = std::fmin(std::fmax(y, -hi), hi);
      q[b * block + i] = f32_to_e4m3(y);
    }
    scales[b] = std::ldexp(1.0f, e);
  }
}

void unpack_host(const uint8_t* q, const float* scales, int64_t n, uint16_t* out, int block) {
  for (int64_t i = 0; i < n; ++i) out[i] = f32_to_bf16(e4m3_to_f32(q[i]) * scales[i / block]);
}

void pack_layer_host(const uint8_t* src, int64_t src_bytes, int64_t src_chunk, int block, uint8_t* dst) {
  check(src_bytes, src_chunk, block);
  for (int64_t off = 0; off < src_bytes; off += src_chunk) {
    const int64_t len = std::min(src_chunk, src_bytes - off);
    const int64_t n = len / 2;
    uint8_t* out = dst + (off / src_chunk) * packed_chunk(src_chunk, block);
    pack_host(reinterpret_cast<const uint16_t*>(src + off), n, out, reinterpret_cast<float*>(out + n), block);
  }
}

void unpack_layer_host(const uint8_t* packed, int64_t src_bytes, int64_t src_chunk, int block, uint8_t* dst) {
  check(src_bytes, src_chunk, block);
  for (int64_t off = 0; off < src_bytes; off += src_chunk) {
    const int64_t len = std::min(src_chunk, src_bytes - off);
    const int64_t n = len / 2;
    const uint8_t* in = packed + (off / src_chunk) * packed_chunk(src_chunk, block);
    unpack_host(in, reinterpret_cast<const float*>(in + n), n, reinterpret_cast<uint16_t*>(dst + off), block);
  }
}

}  // namespace fp8
}  // namespace dissem
