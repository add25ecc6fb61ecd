#include "core/crc32c.h"

#include <mutex>

namespace dissem {

namespace {
uint32_t g_t0[256];
uint32_t g_t16[16 * 256];
uint32_t g_x2n[64];  // x^(2^k) mod P
std::once_flag g_once;

void init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrc32cPoly : c >> 1;
    g_t0[i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i) g_t16[i] = g_t0[i];
  for (int k = 1; k < 16; ++k)
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t prev = g_t16[(k - 1) * 256 + i];
      g_t16[k * 256 + i] = (prev >> 8) ^ g_t0[prev & 0xFF];
    }
  uint32_t p = 1u << 30;  // x^1
  g_x2n[0] = p;
  for (int k = 1; k < 64; ++k) g_x2n[k] = p = crc32c_multmodp(p, p);
}
}  // namespace

uint32_t crc32c_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kCrc32cPoly : b >> 1;
    if (!m) break;
  }
  return p;
}

uint32_t crc32c_xpow8n(uint64_t nbytes) {
  std::call_once(g_once, init_tables);
  uint32_t p = 1u << 31;  // x^0
  uint64_t n = nbytes;
  int k = 3;              // 8 * n = n * 2^3
  while (n) {
    if (n & 1) p = crc32c_multmodp(g_x2n[k & 63], p);
    n >>= 1;
    ++k;
  }
  return p;
}

uint32_t crc32c_raw(const void* data, size_t n, uint32_t crc) {
  std::call_once(g_once, init_tables);
  auto* p = static_cast<const uint8_t*>(data);
  while (n >= 16) {
    uint32_t w0 = uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
    w0 ^= crc;
    crc = g_t16[15 * 256 + (w0 & 0xFF)] ^ g_t16[14 * 256 + ((w0 >> 8) & 0xFF)] ^
          g_t16[13 * 256 + ((w0 >> 16) & 0xFF)] ^ g_t16[12 * 256 + (w0 >> 24)];
    for (int i = 4; i < 16; ++i) crc ^= g_t16[(15 - i) * 256 + p[i]];
    p += 16;
    n -= 16;
  }
  while (n--) crc = g_t0[(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return crc;
}

uint32_t crc32c(const void* data, size_t n, uint32_t crc) {
  return crc32c_raw(data, n, crc ^ 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

void crc32c_slice16_tables(uint32_t* T) {
  std::call_once(g_once, init_tables);
  for (int i = 0; i < 16 * 256; ++i) T[i] = g_t16[i];
}

void crc32c_shift_tables(uint64_t nbytes, uint32_t* A) {
  uint32_t x = crc32c_xpow8n(nbytes);
  for (int b = 0; b < 4; ++b)
    for (uint32_t v = 0; v < 256; ++v) A[b * 256 + v] = v ? crc32c_multmodp(x, v << (8 * b)) : 0;
}

}  // namespace dissem
