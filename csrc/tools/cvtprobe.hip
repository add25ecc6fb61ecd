// cvtprobe: what gfx950's scaled fp8 conversions compute (ISA semantics probe).
// Prints, for a few fp8 codes and scales, the bf16 results of
// v_cvt_scalef32_pk_bf16_fp8 next to code * scale, and the fp8 codes that
// v_cvt_scalef32_pk_fp8_bf16 produces for bf16 inputs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

__global__ void unpack_probe(const int* codes, const float* scales, int n, uint32_t* out) {
  const int i = threadIdx.x;
  if (i >= n) return;
  bf16x2 r = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(codes[i], scales[i], false);
  out[i] = __builtin_bit_cast(uint32_t, r);
}

__global__ void pack_probe(const uint32_t* bf16pairs, const float* scales, int n, uint32_t* out) {
  const int i = threadIdx.x;
  if (i >= n) return;
  i16x2 old = {0, 0};
  auto r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(old, __builtin_bit_cast(bf16x2, bf16pairs[i]), scales[i], false);
  out[i] = uint32_t(__builtin_bit_cast(uint32_t, r));
}

static float bf16f(uint16_t b) {
  uint32_t u = uint32_t(b) << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static uint16_t fbf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return uint16_t(u >> 16);
}

int main() {
  // fp8 e4m3fn codes: 0x38 = 1.0, 0x40 = 2.0, 0x7E = 448, 0x01 = 2^-9 (subnormal)
  const int n = 8;
  int codes[n] = {0x3838, 0x4038, 0x7E38, 0x0138, 0x3838, 0x3838, 0x3838, 0x3838};
  float scales[n] = {1.0f, 1.0f, 1.0f, 1.0f, 3.0f, 0.75f, 1024.0f, 1.5f};
  int *dc;
  float* ds;
  uint32_t* dout;
  hipMalloc(&dc, sizeof codes);
  hipMalloc(&ds, sizeof scales);
  hipMalloc(&dout, n * 4);
  hipMemcpy(dc, codes, sizeof codes, hipMemcpyHostToDevice);
  hipMemcpy(ds, scales, sizeof scales, hipMemcpyHostToDevice);
  unpack_probe<<<1, 64>>>(dc, ds, n, dout);
  uint32_t out[n];
  hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i)
    printf("{\"op\": \"unpack\", \"codes\": \"0x%04x\", \"scale\": %g, \"lo\": %g, \"hi\": %g}\n", codes[i] & 0xFFFF,
           scales[i], bf16f(uint16_t(out[i] & 0xFFFF)), bf16f(uint16_t(out[i] >> 16)));
  uint32_t pairs[n];
  float vals[n][2] = {{1.0f, 2.0f}, {448.0f, -448.0f}, {3.0f, 5.0f}, {1000.0f, 0.1f},
                      {1.0f, 2.0f}, {1.0f, 2.0f}, {1.0f, 2.0f}, {1.0f, 2.0f}};
  float pscales[n] = {1.0f, 1.0f, 1.0f, 1.0f, 2.0f, 3.0f, 0.5f, 1.5f};
  for (int i = 0; i < n; ++i) pairs[i] = uint32_t(fbf16(vals[i][0])) | (uint32_t(fbf16(vals[i][1])) << 16);
  uint32_t* dp;
  hipMalloc(&dp, sizeof pairs);
  hipMemcpy(dp, pairs, sizeof pairs, hipMemcpyHostToDevice);
  hipMemcpy(ds, pscales, sizeof pscales, hipMemcpyHostToDevice);
  pack_probe<<<1, 64>>>(dp, ds, n, dout);
  hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i)
    printf("{\"op\": \"pack\", \"in\": [%g, %g], \"scale\": %g, \"codes\": \"0x%04x\"}\n", vals[i][0], vals[i][1],
           pscales[i], out[i] & 0xFFFF);
  return 0;
}
