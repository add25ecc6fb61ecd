// gfx950 device helper shared by the fp8 kernels (fp8.hip, crc32c.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dissem {
namespace kern {

// Two OCP e4m3fn codes (bytes 0-1 of `w`, or bytes 2-3 if HI) times the
// power-of-two block scale `s` -> two bf16 (first value in the low half):
// v_cvt_scalef32_pk_bf16_fp8, one VALU per pair. The instruction applies only
// the exponent of `s` (an E8M0 scale; profiles/r3_cvt), which is all a
// core/fp8.h scale has, so the product is exact.
template <bool HI>
__device__ __forceinline__ uint32_t fp8x2_to_bf16x2(uint32_t w, float s) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(int(w), s, HI));
}

}  // namespace kern
}  // namespace dissem
