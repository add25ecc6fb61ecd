// Random layer payloads (BASELINE: "synthetic dummy-layer payloads of the
// configured LayerSize filled with random bytes"; the reference fills zeros,
// cmd/config.go:141,161).
//
// Counter-based: u64 word j of the stream = splitmix64(seed + (j+1)*golden).
// Memory-bound: each lane stores 16 B (two words) per iteration, grid-strided
// over ~8 blocks/CU so the store stream saturates HBM.
#include <hip/hip_runtime.h>

#include "kernels/kernels.h"

namespace dissem {
namespace kern {

__host__ __device__ inline uint64_t mix64(uint64_t seed, uint64_t j) {
  uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) fill_random_kernel(ulonglong2* __restrict__ dst, int64_t nvec,
                                                          uint64_t seed) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    // one 16-B nontemporal store per lane: whole lines per instruction (two 8-B
    // stores leave each instruction's lines half written, which NT stores pay
    // for: profiles/r4_nt, store 14)
    using v2u64 = unsigned long long __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(v2u64{mix64(seed, uint64_t(2 * i)), mix64(seed, uint64_t(2 * i + 1))},
                                reinterpret_cast<v2u64*>(dst) + i);
  }
}

__global__ void fill_tail_kernel(uint8_t* __restrict__ dst, int64_t first, int64_t bytes, uint64_t seed) {
  int64_t b = first + threadIdx.x;
  if (b >= bytes) return;
  uint64_t w = mix64(seed, uint64_t(b >> 3));
  dst[b] = uint8_t(w >> (8 * (b & 7)));
}

hipError_t fill_random(void* dst, int64_t bytes, uint64_t seed, hipStream_t s) {
  if (bytes <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(dst) & 15) return hipErrorInvalidValue;
  int64_t nvec = bytes / 16;
  if (nvec) {
    int64_t blocks = (nvec + 255) / 256;
    if (blocks > 2048) blocks = 2048;  // 8 per CU, grid-stride the rest
    fill_random_kernel<<<dim3(unsigned(blocks)), dim3(256), 0, s>>>(static_cast<ulonglong2*>(dst), nvec, seed);
  }
  if (bytes % 16)
    fill_tail_kernel<<<1, 64, 0, s>>>(static_cast<uint8_t*>(dst), nvec * 16, bytes, seed);
  return hipGetLastError();
}

void fill_random_host(void* dst, int64_t bytes, uint64_t seed, int64_t offset) {
  // Bytes [offset, offset+bytes) of the stream (offset: any byte position).
  auto* p = static_cast<uint8_t*>(dst);
  for (int64_t i = 0; i < bytes;) {
    const int64_t b = offset + i;
    if ((b & 7) == 0 && bytes - i >= 8) {
      uint64_t w = mix64(seed, uint64_t(b >> 3));
      for (int k = 0; k < 8; ++k) p[i + k] = uint8_t(w >> (8 * k));
      i += 8;
    } else {
      p[i] = uint8_t(mix64(seed, uint64_t(b >> 3)) >> (8 * (b & 7)));
      ++i;
    }
  }
}

// Test helper: one wave that holds its stream until the host sets `flag`
// (host-mapped, coherent) or max_iters sleeps have passed - a stand-in for an
// RCCL kernel waiting on a peer. Always exits; writes how long it waited.
__global__ void __launch_bounds__(64) spin_until_kernel(const volatile uint32_t* flag, uint64_t max_iters,
                                                         uint64_t* iters) {
  if (threadIdx.x != 0) return;
  uint64_t i = 0;
  while (i < max_iters && *flag == 0) {
    __builtin_amdgcn_s_sleep(127);
    ++i;
  }
  *iters = i;
}

hipError_t spin_until(const uint32_t* flag, uint64_t max_iters, uint64_t* iters, hipStream_t s) {
  spin_until_kernel<<<dim3(1), dim3(64), 0, s>>>(flag, max_iters, iters);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace dissem
