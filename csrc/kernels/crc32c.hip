// Per-chunk CRC32C on gfx950 (receiver-side verification of every landed chunk).
//
// CRC is a serial recurrence, so the kernel works with raw (un-inverted) CRC
// registers, which are linear over GF(2):
//   raw(A || B) = shift(raw(A), |B|) xor raw(B),  shift(r, L) = r * x^(8L) mod P.
// Decomposition:
//  * a chunk is cut into 16 KiB segments; one wave owns a segment;
//  * lane l of the wave reads 16-B words l, l+64, l+128, ... (each wave
//    instruction reads 1 KiB contiguous: fully coalesced) and keeps the raw CRC
//    of its strided sub-message: s = shift_1024B(s) xor crc16(word), i.e. 4 + 16
//    table lookups from LDS-resident slice-by-16 and shift tables;
//  * lanes are aligned to the segment end with one GF(2) multiply by a per-lane
//    constant x^(8*16*m) and XOR-reduced with cross-lane shuffles;
//  * a second, tiny kernel folds the segments of each chunk (one wave per
//    chunk) and applies the init/xorout term, writing the standard CRC32C.
// The result is the exact CRC32C of each chunk for any chunk length that is a
// multiple of 16 (the final chunk may have any length).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <vector>

#include "core/crc32c.h"
#include "kernels/kernels.h"

namespace dissem {
namespace kern {

namespace {

// 16 KiB per wave: 16 strided words per lane. Small enough that one 64 MiB
// landing chunk spreads over 4096 waves (16 per CU), large enough that the
// per-wave lane-alignment multiply is amortized.
constexpr int kSegBytes = 16 * 1024;
constexpr int kT16 = 16 * 256;   // slice-by-16 tables
constexpr int kA = 4 * 256;      // shift-by-1024-bytes map
constexpr int kLanePow = 64;     // x^(8*16*m), m = 0..63
constexpr int kAS = 4 * 256;     // shift-by-one-segment map
constexpr int kX2N = 64;         // x^(2^k)
constexpr int kConstWords = kT16 + kA + kLanePow + kAS + kX2N;
constexpr int kSegKernelLds = kT16 + kA + kLanePow;

__device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 1
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    b = (b & 1) ? (b >> 1) ^ kCrc32cPoly : b >> 1;
  }
  return p;
}

__device__ inline uint32_t xpow8n(const uint32_t* x2n, uint64_t n) {
  uint32_t p = 1u << 31;
  int k = 3;
#pragma unroll 1
  while (n) {
    if (n & 1) p = multmodp(x2n[k & 63], p);
    n >>= 1;
    ++k;
  }
  return p;
}

__device__ inline uint32_t shift_map(const uint32_t* A, uint32_t s) {
  return A[s & 255] ^ A[256 + ((s >> 8) & 255)] ^ A[512 + ((s >> 16) & 255)] ^ A[768 + (s >> 24)];
}

__device__ inline uint32_t crc16raw(const uint32_t* T, uint4 w) {
  return T[15 * 256 + (w.x & 255)] ^ T[14 * 256 + ((w.x >> 8) & 255)] ^ T[13 * 256 + ((w.x >> 16) & 255)] ^
         T[12 * 256 + (w.x >> 24)] ^ T[11 * 256 + (w.y & 255)] ^ T[10 * 256 + ((w.y >> 8) & 255)] ^
         T[9 * 256 + ((w.y >> 16) & 255)] ^ T[8 * 256 + (w.y >> 24)] ^ T[7 * 256 + (w.z & 255)] ^
         T[6 * 256 + ((w.z >> 8) & 255)] ^ T[5 * 256 + ((w.z >> 16) & 255)] ^ T[4 * 256 + (w.z >> 24)] ^
         T[3 * 256 + (w.w & 255)] ^ T[2 * 256 + ((w.w >> 8) & 255)] ^ T[1 * 256 + ((w.w >> 16) & 255)] ^
         T[0 * 256 + (w.w >> 24)];
}

__device__ inline uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}

// One wave per 16 KiB segment; writes the segment's raw CRC to seg_out[g].
__global__ void __launch_bounds__(256) crc32c_segments_kernel(const uint8_t* __restrict__ src, int64_t bytes,
                                                              int64_t chunk_bytes, int64_t spc,
                                                              int64_t total_segs,
                                                              const uint32_t* __restrict__ consts,
                                                              uint32_t* __restrict__ seg_out) {
  __shared__ uint32_t lds[kSegKernelLds];
  for (int i = threadIdx.x; i < kSegKernelLds; i += blockDim.x) lds[i] = consts[i];
  __syncthreads();
  const uint32_t* T = lds;
  const uint32_t* A = lds + kT16;
  const uint32_t* lanepow = lds + kT16 + kA;

  const int lane = threadIdx.x & 63;
  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x / 64);
  for (int64_t g = wave; g < total_segs; g += nwaves) {
    const int64_t c = g / spc, k = g % spc;
    const int64_t chunk_start = c * chunk_bytes;
    const int64_t chunk_len = min(chunk_bytes, bytes - chunk_start);
    const int64_t seg_start = k * kSegBytes;
    const int64_t seg_len = min(int64_t(kSegBytes), chunk_len - seg_start);
    const int64_t nw = seg_len >> 4;
    const uint4* words = reinterpret_cast<const uint4*>(src + chunk_start + seg_start);
    uint32_t s = 0;
    int64_t j = lane;
    if (nw == kSegBytes / 16) {
      // Full segment: 64 words per lane, loads issued 8 ahead.
#pragma unroll 8
      for (int it = 0; it < kSegBytes / 16 / 64; ++it) {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        const u32x4 wv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(words + lane + 64 * it));
        const uint4 w = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        s = shift_map(A, s) ^ crc16raw(T, w);
      }
      s = multmodp(lanepow[63 - lane], s);
    } else {
      int64_t last = -1;
      for (; j < nw; j += 64) {
        uint4 w = words[j];
        s = shift_map(A, s) ^ crc16raw(T, w);
        last = j;
      }
      if (last >= 0) s = multmodp(lanepow[nw - 1 - last], s);
    }
    s = wave_xor(s);
    if (lane == 0) {
      // Byte tail (only the buffer's final segment can have one).
      const uint8_t* tail = src + chunk_start + seg_start + (nw << 4);
      for (int64_t b = 0; b < (seg_len & 15); ++b) s = T[(s ^ tail[b]) & 255] ^ (s >> 8);
      seg_out[g] = s;
    }
  }
}

__device__ inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return uint16_t((u >> 16) | 0x40);  // quiet NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

// 16 e4m3fn values (one 16-B word) times their block scale -> 16 bf16 (two 16-B words).
__device__ inline void unpack16(uint4 w, float s, uint4* __restrict__ dst) {
  const uint32_t d[4] = {w.x, w.y, w.z, w.w};
  uint32_t o[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(int(d[i]), false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(int(d[i]), true);
    o[2 * i] = uint32_t(f32_to_bf16_rne(lo[0] * s)) | (uint32_t(f32_to_bf16_rne(lo[1] * s)) << 16);
    o[2 * i + 1] = uint32_t(f32_to_bf16_rne(hi[0] * s)) | (uint32_t(f32_to_bf16_rne(hi[1] * s)) << 16);
  }
  dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
  dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// Fused verify + unpack of fp8-packed chunks (core/fp8.h layout
// [q: n bytes][scales: n/BLOCK f32] per chunk): one pass over the packed bytes
// computes each segment's raw CRC exactly like crc32c_segments_kernel and, for
// words in the q region, writes the dequantized bf16 values. Every packed byte
// is read once from HBM; the scales (1/32 of the traffic) are re-read from L2.
template <int BLOCK>
__global__ void __launch_bounds__(256) verify_unpack_segments_kernel(
    const uint8_t* __restrict__ src, int64_t bytes, int64_t pchunk, int64_t spc, int64_t total_segs,
    int64_t out_chunk_elems, const uint32_t* __restrict__ consts, uint32_t* __restrict__ seg_out,
    uint16_t* __restrict__ out) {
  __shared__ uint32_t lds[kSegKernelLds];
  for (int i = threadIdx.x; i < kSegKernelLds; i += blockDim.x) lds[i] = consts[i];
  __syncthreads();
  const uint32_t* T = lds;
  const uint32_t* A = lds + kT16;
  const uint32_t* lanepow = lds + kT16 + kA;

  const int lane = threadIdx.x & 63;
  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x / 64);
  for (int64_t g = wave; g < total_segs; g += nwaves) {
    const int64_t c = g / spc, k = g % spc;
    const int64_t chunk_start = c * pchunk;
    const int64_t chunk_len = min(pchunk, bytes - chunk_start);
    const int64_t n_q = chunk_len / (BLOCK + 4) * BLOCK;  // q bytes (= elements) of this chunk
    const float* scales = reinterpret_cast<const float*>(src + chunk_start + n_q);
    uint16_t* obase = out + c * out_chunk_elems;
    const int64_t seg_start = k * kSegBytes;
    const int64_t seg_len = min(int64_t(kSegBytes), chunk_len - seg_start);
    const int64_t nw = seg_len >> 4;
    const uint4* words = reinterpret_cast<const uint4*>(src + chunk_start + seg_start);
    uint32_t s = 0;
    auto consume = [&](const uint4 w, int64_t j) {
      s = shift_map(A, s) ^ crc16raw(T, w);
      const int64_t e = seg_start + 16 * j;  // byte offset in chunk = element index in the q region
      if (e < n_q) unpack16(w, scales[e / BLOCK], reinterpret_cast<uint4*>(obase + e));
    };
    if (nw == kSegBytes / 16) {
#pragma unroll 8
      for (int it = 0; it < kSegBytes / 16 / 64; ++it) {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        const u32x4 wv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(words + lane + 64 * it));
        consume(make_uint4(wv[0], wv[1], wv[2], wv[3]), lane + 64 * it);
      }
      s = multmodp(lanepow[63 - lane], s);
    } else {
      int64_t last = -1;
      for (int64_t j = lane; j < nw; j += 64) {
        consume(words[j], j);
        last = j;
      }
      if (last >= 0) s = multmodp(lanepow[nw - 1 - last], s);
    }
    s = wave_xor(s);
    if (lane == 0) {
      const uint8_t* tail = src + chunk_start + seg_start + (nw << 4);
      for (int64_t b = 0; b < (seg_len & 15); ++b) s = T[(s ^ tail[b]) & 255] ^ (s >> 8);
      seg_out[g] = s;
    }
  }
}

// One wave per chunk: fold the chunk's segment CRCs and finalize. `fold` holds
// host-computed constants for full chunks: per lane x^(8*bytes after its run)
// and the init/xorout term; only a short final chunk computes them here.
__global__ void __launch_bounds__(64) crc32c_fold_kernel(const uint32_t* __restrict__ seg_out, int64_t bytes,
                                                         int64_t chunk_bytes, int64_t spc,
                                                         const uint32_t* __restrict__ consts,
                                                         const uint32_t* __restrict__ fold,
                                                         uint32_t* __restrict__ out) {
  __shared__ uint32_t AS[kAS];
  __shared__ uint32_t X2N[kX2N];
  for (int i = threadIdx.x; i < kAS; i += 64) AS[i] = consts[kT16 + kA + kLanePow + i];
  for (int i = threadIdx.x; i < kX2N; i += 64) X2N[i] = consts[kT16 + kA + kLanePow + kAS + i];
  __syncthreads();
  const int lane = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t chunk_start = c * chunk_bytes;
  const int64_t chunk_len = min(chunk_bytes, bytes - chunk_start);
  const int64_t n = (chunk_len + kSegBytes - 1) / kSegBytes;
  const int64_t q = (n + 63) / 64;
  const int64_t b = min(n, int64_t(lane) * q), e = min(n, int64_t(lane + 1) * q);
  uint32_t r = 0;
  for (int64_t k = b; k < e; ++k) {
    const int64_t len = min(int64_t(kSegBytes), chunk_len - k * kSegBytes);
    r = (len == kSegBytes ? shift_map(AS, r) : multmodp(xpow8n(X2N, uint64_t(len)), r)) ^ seg_out[c * spc + k];
  }
  const bool full = chunk_len == chunk_bytes;
  const int64_t end_byte = min(e * kSegBytes, chunk_len);
  if (r && e > b) r = multmodp(full ? fold[lane] : xpow8n(X2N, uint64_t(chunk_len - end_byte)), r);
  r = wave_xor(e > b ? r : 0u);
  if (lane == 0)
    out[c] = r ^ (full ? fold[64] : (multmodp(xpow8n(X2N, uint64_t(chunk_len)), 0xFFFFFFFFu) ^ 0xFFFFFFFFu));
}

struct DeviceConsts {
  std::mutex mu;
  std::map<int, uint32_t*> by_device;
  std::map<std::pair<int, int64_t>, uint32_t*> fold;  // (device, chunk_bytes) -> 65 fold constants
};
DeviceConsts g_consts;

uint32_t* fold_consts(int64_t chunk_bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_consts.mu);
  auto key = std::make_pair(dev, chunk_bytes);
  auto it = g_consts.fold.find(key);
  if (it != g_consts.fold.end()) return it->second;
  const int64_t n = (chunk_bytes + kSegBytes - 1) / kSegBytes, q = (n + 63) / 64;
  std::vector<uint32_t> h(65);
  for (int l = 0; l < 64; ++l) {
    int64_t e = std::min(n, int64_t(l + 1) * q);
    int64_t end_byte = std::min(e * kSegBytes, chunk_bytes);
    h[size_t(l)] = crc32c_xpow8n(uint64_t(chunk_bytes - end_byte));
  }
  h[64] = crc32c_init_term(uint64_t(chunk_bytes));
  uint32_t* d = nullptr;
  if (hipMalloc(&d, h.size() * 4) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  g_consts.fold[key] = d;
  return d;
}

uint32_t* device_consts() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_consts.mu);
  auto it = g_consts.by_device.find(dev);
  if (it != g_consts.by_device.end()) return it->second;
  std::vector<uint32_t> h(kConstWords);
  crc32c_slice16_tables(h.data());
  crc32c_shift_tables(1024, h.data() + kT16);
  for (int m = 0; m < 64; ++m) h[size_t(kT16 + kA + m)] = crc32c_xpow8n(uint64_t(16) * uint64_t(m));
  crc32c_shift_tables(kSegBytes, h.data() + kT16 + kA + kLanePow);
  uint32_t p = 1u << 30;
  for (int k = 0; k < 64; ++k) {
    h[size_t(kT16 + kA + kLanePow + kAS + k)] = p;
    p = crc32c_multmodp(p, p);
  }
  uint32_t* d = nullptr;
  if (hipMalloc(&d, h.size() * 4) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  g_consts.by_device[dev] = d;
  return d;
}

}  // namespace

size_t crc32c_workspace_bytes(int64_t bytes, int64_t chunk_bytes) {
  if (bytes <= 0 || chunk_bytes <= 0) return 16;
  int64_t spc = (chunk_bytes + kSegBytes - 1) / kSegBytes;
  int64_t nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  return size_t(nchunks * spc * 4 + 16);
}

hipError_t crc32c_chunks(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                         hipStream_t s) {
  if (bytes <= 0) return hipSuccess;
  if (chunk_bytes <= 0 || chunk_bytes % 16 || (reinterpret_cast<uintptr_t>(src) & 15)) return hipErrorInvalidValue;
  uint32_t* consts = device_consts();
  uint32_t* fold = fold_consts(chunk_bytes);
  if (!consts || !fold) return hipErrorOutOfMemory;
  const int64_t spc = (chunk_bytes + kSegBytes - 1) / kSegBytes;
  const int64_t nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  const int64_t last_len = bytes - (nchunks - 1) * chunk_bytes;
  const int64_t total_segs = (nchunks - 1) * spc + (last_len + kSegBytes - 1) / kSegBytes;
  int64_t blocks = (total_segs + 3) / 4;
  if (blocks > 256 * 6) blocks = 256 * 6;
  auto* seg = static_cast<uint32_t*>(workspace);
  crc32c_segments_kernel<<<dim3(unsigned(blocks)), dim3(256), 0, s>>>(static_cast<const uint8_t*>(src), bytes,
                                                                      chunk_bytes, spc, total_segs, consts, seg);
  crc32c_fold_kernel<<<dim3(unsigned(nchunks)), dim3(64), 0, s>>>(seg, bytes, chunk_bytes, spc, consts, fold, out);
  return hipGetLastError();
}

hipError_t fp8_verify_unpack(const void* packed, int64_t src_bytes, int64_t src_chunk, int block, uint16_t* out,
                             uint32_t* crc_out, void* workspace, hipStream_t s) {
  if (src_bytes <= 0) return hipSuccess;
  if (src_chunk <= 0 || src_chunk % 4096 || src_bytes % (2 * block) || (reinterpret_cast<uintptr_t>(packed) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 15))
    return hipErrorInvalidValue;
  const int64_t pchunk = src_chunk / 2 + src_chunk / 2 / block * 4;
  const int64_t full = src_bytes / src_chunk, tail = src_bytes % src_chunk;
  const int64_t bytes = full * pchunk + (tail ? tail / 2 + tail / 2 / block * 4 : 0);
  uint32_t* consts = device_consts();
  uint32_t* fold = fold_consts(pchunk);
  if (!consts || !fold) return hipErrorOutOfMemory;
  const int64_t spc = (pchunk + kSegBytes - 1) / kSegBytes;
  const int64_t nchunks = (bytes + pchunk - 1) / pchunk;
  const int64_t last_len = bytes - (nchunks - 1) * pchunk;
  const int64_t total_segs = (nchunks - 1) * spc + (last_len + kSegBytes - 1) / kSegBytes;
  int64_t blocks = (total_segs + 3) / 4;
  if (blocks > 256 * 6) blocks = 256 * 6;
  auto* seg = static_cast<uint32_t*>(workspace);
  auto* p = static_cast<const uint8_t*>(packed);
  const dim3 grid{unsigned(blocks)}, tpb{256};
  switch (block) {
    case 32: verify_unpack_segments_kernel<32><<<grid, tpb, 0, s>>>(p, bytes, pchunk, spc, total_segs, src_chunk / 2, consts, seg, out); break;
    case 64: verify_unpack_segments_kernel<64><<<grid, tpb, 0, s>>>(p, bytes, pchunk, spc, total_segs, src_chunk / 2, consts, seg, out); break;
    case 128: verify_unpack_segments_kernel<128><<<grid, tpb, 0, s>>>(p, bytes, pchunk, spc, total_segs, src_chunk / 2, consts, seg, out); break;
    case 256: verify_unpack_segments_kernel<256><<<grid, tpb, 0, s>>>(p, bytes, pchunk, spc, total_segs, src_chunk / 2, consts, seg, out); break;
    case 512: verify_unpack_segments_kernel<512><<<grid, tpb, 0, s>>>(p, bytes, pchunk, spc, total_segs, src_chunk / 2, consts, seg, out); break;
    default: return hipErrorInvalidValue;
  }
  crc32c_fold_kernel<<<dim3(unsigned(nchunks)), dim3(64), 0, s>>>(seg, bytes, pchunk, spc, consts, fold, crc_out);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace dissem
