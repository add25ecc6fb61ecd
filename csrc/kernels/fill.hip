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

// Read roofline probe: every byte read once (16 B per lane, `depth` loads in
// flight per lane, grid-stride), XOR-folded to one dword per wave so the loads
// cannot be elided. The bound a read-only verify kernel could reach with the
// same access pattern.
template <int DEPTH>
__global__ void __launch_bounds__(256) read_xor_kernel(const uint4* __restrict__ src, int64_t nvec,
                                                       uint32_t* __restrict__ out) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  uint32_t acc = 0;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
  for (; i + (DEPTH - 1) * stride < nvec; i += DEPTH * stride) {
    u32x4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) v[d] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i + d * stride));
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) acc ^= v[d][0] ^ v[d][1] ^ v[d][2] ^ v[d][3];
  }
  for (; i < nvec; i += stride) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  for (int o = 32; o > 0; o >>= 1) acc ^= uint32_t(__shfl_xor(int(acc), o, 64));
  if ((threadIdx.x & 63) == 0) out[(int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6] = acc;
}

hipError_t read_xor(const void* src, int64_t bytes, uint32_t* out, int blocks, int depth, hipStream_t s) {
  if (bytes <= 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(src) & 15) || bytes % 16 || blocks <= 0) return hipErrorInvalidValue;
  const auto* p = static_cast<const uint4*>(src);
  switch (depth) {
    case 1: read_xor_kernel<1><<<dim3(unsigned(blocks)), dim3(256), 0, s>>>(p, bytes / 16, out); break;
    case 2: read_xor_kernel<2><<<dim3(unsigned(blocks)), dim3(256), 0, s>>>(p, bytes / 16, out); break;
    case 8: read_xor_kernel<8><<<dim3(unsigned(blocks)), dim3(256), 0, s>>>(p, bytes / 16, out); break;
    default: read_xor_kernel<4><<<dim3(unsigned(blocks)), dim3(256), 0, s>>>(p, bytes / 16, out); break;
  }
  return hipGetLastError();
}

// Segment-read probe: the CRC kernels' access shape with no compute. One wave
// reads one 16 KiB segment at a time (16 x 16-B loads per lane, all in flight),
// grid-strided over segments, 1024-thread workgroups. layout 0: lane l takes
// the 64-B piece l of each 4 KiB block (crc32c v3); 1: the 16-B words l + 64 i
// (v1/v2). rolling: the next segment's word i is loaded as word i is consumed.
template <int LAYOUT, bool ROLL>
__global__ void __launch_bounds__(1024) read_seg_kernel(const uint8_t* __restrict__ src, int64_t nseg,
                                                        uint32_t* __restrict__ out) {
  using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int64_t wave = int64_t(blockIdx.x) * 16 + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * 16;
  auto at = [&](int64_t g, int i) {
    const uint8_t* seg = src + g * 16384;
    return reinterpret_cast<const u32x4*>(LAYOUT == 0 ? seg + (i >> 2) * 4096 + 64 * lane + 16 * (i & 3)
                                                      : seg + 16 * (lane + 64 * i));
  };
  uint32_t acc = 0;
  u32x4 w[16];
  int64_t g = wave;
  if (g < nseg) {
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = __builtin_nontemporal_load(at(g, i));
  }
  for (; g < nseg; g += nwaves) {
    const int64_t gn = g + nwaves;
    if (ROLL && gn < nseg) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const u32x4 x = w[i];
        acc ^= x[0] ^ x[1] ^ x[2] ^ x[3];
        w[i] = __builtin_nontemporal_load(at(gn, i));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= w[i][0] ^ w[i][1] ^ w[i][2] ^ w[i][3];
      if (gn < nseg) {
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = __builtin_nontemporal_load(at(gn, i));
      }
    }
  }
  out[int64_t(blockIdx.x) * blockDim.x + threadIdx.x] = acc;
}

hipError_t read_seg(const void* src, int64_t bytes, uint32_t* out, int blocks, int layout, bool roll, hipStream_t s) {
  if (bytes <= 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(src) & 15) || bytes % 16384 || blocks <= 0) return hipErrorInvalidValue;
  const auto* p = static_cast<const uint8_t*>(src);
  const int64_t nseg = bytes / 16384;
  const dim3 g{unsigned(blocks)}, b{1024};
  if (layout == 0) {
    if (roll) read_seg_kernel<0, true><<<g, b, 0, s>>>(p, nseg, out);
    else read_seg_kernel<0, false><<<g, b, 0, s>>>(p, nseg, out);
  } else {
    if (roll) read_seg_kernel<1, true><<<g, b, 0, s>>>(p, nseg, out);
    else read_seg_kernel<1, false><<<g, b, 0, s>>>(p, nseg, out);
  }
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
