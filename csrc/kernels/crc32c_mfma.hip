// CRC32C on the matrix cores: a GF(2) matrix-vector product per 64-B block,
// computed with v_mfma_i32_32x32x32_i8 and reduced mod 2.
//
// The raw CRC of a 64-byte block (zero register) is linear in its 512 bits:
//   crc(block) = M * bits(block) over GF(2),  M: 32 x 512, column i = crc(e_i).
// For 32 blocks at once that is D = M * X with X = [bits of block 0 .. 31]
// (512 x 32): an int8 GEMM with 0/1 entries whose int32 results, taken mod 2,
// are the 32 CRC bits of each block. M (16 K-steps of 32x32 int8) lives in the
// wave's registers for the whole kernel; X comes straight from the loaded
// words: bit-plane p of a dword w is (w >> p) & 0x01010101 - four 0/1 bytes
// per VALU pair - so one K-step costs ~8 VALU + 1 MFMA per lane for 128 B.
//
// The K order inside a fragment does not matter as long as A and B agree:
// element j = 4t + b (VGPR t, byte b) of lane half h stands for bit
// 8b + 4h + t of dword s of the block, in both operands. D's layout is the
// documented 32x32 map (col = lane & 31, row = (reg&3) + 8(reg>>2) + 4(lane>>5)).
//
// Blocks are chained exactly like the nibble-table kernel chains words: lane n
// of a wave owns blocks n, n+32, ..., n+224 of a 16 KiB segment (2 KiB apart):
// s = shift_2KiB(s) xor crc(block), the shift via 8 bank-private nibble tables
// in LDS (16 KiB); then one GF(2) multiply per lane shifts its CRC to the end
// of its chunk and the 32 lanes are XOR-reduced. The fold kernel is shared
// with crc32c.hip (seg_out holds chunk-end-shifted segment CRCs).
//
// Applies to chunk lengths that are whole 16 KiB segments. Reached through
// crc32c_chunks_impl (kMfma, or kAuto with DISSEM_CRC_IMPL=mfma): that is the
// staging-side verify (HipBackend::crc) and the ops/bindings entry points.
// The batched landing verify (crc32c_batch) and the fused fp8 verify+unpack
// always use the nibble-table kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "core/crc32c.h"
#include "kernels/kernels.h"

namespace dissem {
namespace kern {

namespace {

constexpr int kSeg = 16 * 1024;        // bytes per segment (one wave)
constexpr int kBlock = 64;             // bytes per MFMA column
constexpr int kBatches = kSeg / (32 * kBlock);  // 8 batches of 32 blocks
constexpr int kThreads = 256;
constexpr int kShiftLds = 8 * 16 * 32;  // 8 nibble tables x 16 x 32 replicas (u32)

using v4i = int __attribute__((ext_vector_type(4)));
using v16i = int __attribute__((ext_vector_type(16)));

__device__ inline uint32_t mulmodp(uint32_t a, uint32_t b) {
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

__device__ __forceinline__ uint32_t shift2k(const uint32_t* L, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int n = 0; n < 8; ++n) r ^= L[n * 512 + ((x >> (4 * n)) & 15) * 32];
  return r;
}

// consts layout: [A fragments: 16 steps x 64 lanes x 4 ints][shift-2KiB nibble tables: 8 x 16]
constexpr int kAFragInts = 16 * 64 * 4;

// NACC independent accumulator chains per batch: K-step s accumulates into
// chain s % NACC, so consecutive MFMAs do not wait on each other's result;
// the chains' int32 sums are added before taking bit 0 (parity is additive).
template <int NACC>
__global__ void __launch_bounds__(kThreads) crc32c_mfma_segments_kernel(
    const uint8_t* __restrict__ src, int64_t bytes, int64_t chunk_bytes, int64_t spc, int64_t total_segs,
    const int* __restrict__ consts, const uint32_t* __restrict__ lshift, const uint32_t* __restrict__ lshift_last,
    uint32_t* __restrict__ seg_out) {
  __shared__ uint32_t lds[kShiftLds];
  const uint32_t* nib = reinterpret_cast<const uint32_t*>(consts + kAFragInts);
  for (int i = threadIdx.x; i < kShiftLds / 4; i += blockDim.x) {
    const uint32_t v = nib[i >> 3];
    reinterpret_cast<uint4*>(lds)[i] = make_uint4(v, v, v, v);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5, n = lane & 31;
  const uint32_t* L = lds + n;
  // M in registers: 16 K-steps of this lane's A fragment.
  v4i a[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) a[s] = reinterpret_cast<const v4i*>(consts)[s * 64 + lane];

  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x / 64);
  for (int64_t g = wave; g < total_segs; g += nwaves) {
    const int64_t c = g / spc, k = g % spc;
    const int64_t chunk_start = c * chunk_bytes;
    const int64_t chunk_len = min(chunk_bytes, bytes - chunk_start);
    const uint8_t* seg = src + chunk_start + k * kSeg;
    uint32_t chain = 0;
    using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
    // Two batches in flight per lane: batch b+1's 64 B are requested before
    // batch b's 16 MFMAs issue (the last prefetch re-reads batch 7, an L1 hit).
    const u32x4* blk0 = reinterpret_cast<const u32x4*>(seg + n * kBlock);
    u32x4 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = __builtin_nontemporal_load(blk0 + i);
#pragma unroll 1
    for (int b = 0; b < kBatches; ++b) {
      const int bn = b + 1 < kBatches ? b + 1 : b;
      const u32x4* nblk = reinterpret_cast<const u32x4*>(seg + (32 * bn + n) * kBlock);
      u32x4 qn[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) qn[i] = __builtin_nontemporal_load(nblk + i);
      v16i accs[NACC];
#pragma unroll
      for (int j = 0; j < NACC; ++j) accs[j] = v16i{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const uint32_t w = q[s >> 2][s & 3] >> (4 * h);
        v4i bv;
        bv[0] = int(w & 0x01010101u);
        bv[1] = int((w >> 1) & 0x01010101u);
        bv[2] = int((w >> 2) & 0x01010101u);
        bv[3] = int((w >> 3) & 0x01010101u);
        accs[s % NACC] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], bv, accs[s % NACC], 0, 0, 0);
      }
      v16i acc = accs[0];
#pragma unroll
      for (int j = 1; j < NACC; ++j) acc += accs[j];
      uint32_t part = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) part |= uint32_t(acc[r] & 1) << ((r & 3) + 8 * (r >> 2) + 4 * h);
      const uint32_t crc_block = part | uint32_t(__shfl_xor(int(part), 32, 64));
      chain = shift2k(L, chain) ^ crc_block;
#pragma unroll
      for (int i = 0; i < 4; ++i) q[i] = qn[i];
    }
    // Shift lane n's chain (ends at block 224 + n) to the end of its chunk.
    const uint32_t* row = (chunk_len == chunk_bytes ? lshift : lshift_last) + k * 32;
    uint32_t r = h == 0 ? mulmodp(row[n], chain) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r ^= uint32_t(__shfl_xor(int(r), o, 64));
    if (lane == 0) seg_out[g] = r;
  }
}

struct Tables {
  std::mutex mu;
  std::map<int, int*> consts;
  std::map<std::tuple<int, int64_t, int64_t>, uint32_t*> shifts;  // (dev, chunk, last) -> [spc x 32] x 2
};
Tables g_tab;

int* mfma_consts() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_tab.mu);
  auto it = g_tab.consts.find(dev);
  if (it != g_tab.consts.end()) return it->second;
  // Column i of M: raw CRC of a 64-byte block with only bit i (bit i%8 of byte i/8) set.
  std::vector<uint32_t> col(512);
  for (int i = 0; i < 512; ++i) {
    uint8_t blk[64] = {};
    blk[i / 8] = uint8_t(1u << (i % 8));
    col[size_t(i)] = crc32c_raw(blk, 64, 0);
  }
  std::vector<int> h(size_t(kAFragInts + 8 * 16));
  auto* bytes = reinterpret_cast<int8_t*>(h.data());
  for (int s = 0; s < 16; ++s)
    for (int lane = 0; lane < 64; ++lane) {
      const int r = lane & 31, hh = lane >> 5;
      for (int j = 0; j < 16; ++j) {
        const int t = j / 4, b = j % 4;
        const int bit = 32 * s + 8 * b + 4 * hh + t;
        bytes[(s * 64 + lane) * 16 + j] = int8_t((col[size_t(bit)] >> r) & 1);
      }
    }
  std::vector<uint32_t> A(4 * 256);
  crc32c_shift_tables(2048, A.data());
  auto* nib = reinterpret_cast<uint32_t*>(h.data() + kAFragInts);
  for (int t = 0; t < 8; ++t)
    for (uint32_t v = 0; v < 16; ++v) nib[t * 16 + int(v)] = A[size_t((t / 2) * 256) + (v << (4 * (t & 1)))];
  int* d = nullptr;
  if (hipMalloc(&d, h.size() * 4) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  g_tab.consts[dev] = d;
  return d;
}

// Per segment k of a `len`-byte chunk (len % kSeg == 0) and lane n < 32:
// x^(8 * (64 * (31 - n) + len - (k + 1) * kSeg)).
void lane_shifts32(int64_t len, int64_t spc, uint32_t* out) {
  const int64_t nseg = len / kSeg;
  std::fill(out, out + spc * 32, 0u);
  uint32_t lanepow[32];
  for (int m = 0; m < 32; ++m) lanepow[m] = crc32c_xpow8n(uint64_t(kBlock) * uint64_t(m));
  const uint32_t xs = crc32c_xpow8n(kSeg);
  uint32_t seg = 1u << 31;  // last segment: ends at the chunk end
  for (int64_t k = nseg - 1; k >= 0; --k) {
    for (int l = 0; l < 32; ++l) out[k * 32 + l] = crc32c_multmodp(lanepow[31 - l], seg);
    seg = crc32c_multmodp(xs, seg);
  }
}

uint32_t* mfma_shifts(int64_t chunk, int64_t last) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_tab.mu);
  auto key = std::make_tuple(dev, chunk, last);
  auto it = g_tab.shifts.find(key);
  if (it != g_tab.shifts.end()) return it->second;
  const int64_t spc = chunk / kSeg;
  std::vector<uint32_t> h(size_t(2 * spc * 32));
  lane_shifts32(chunk, spc, h.data());
  lane_shifts32(last, spc, h.data() + spc * 32);
  uint32_t* d = nullptr;
  if (hipMalloc(&d, h.size() * 4) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  g_tab.shifts[key] = d;
  return d;
}

}  // namespace

bool crc32c_mfma_default() {
  static const bool on = [] {
    const char* e = std::getenv("DISSEM_CRC_IMPL");
    return e && std::strcmp(e, "mfma") == 0;
  }();
  return on;
}

bool crc32c_mfma_applies(int64_t bytes, int64_t chunk_bytes) {
  return bytes > 0 && chunk_bytes > 0 && chunk_bytes % kSeg == 0 && bytes % kSeg == 0;
}

hipError_t crc32c_mfma_segments(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* seg_out,
                                hipStream_t s, int max_blocks, int chains) {
  if (!crc32c_mfma_applies(bytes, chunk_bytes) || (reinterpret_cast<uintptr_t>(src) & 15))
    return hipErrorInvalidValue;
  int* consts = mfma_consts();
  const int64_t spc = chunk_bytes / kSeg;
  const int64_t nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  const int64_t last = bytes - (nchunks - 1) * chunk_bytes;
  uint32_t* sh = mfma_shifts(chunk_bytes, last);
  if (!consts || !sh) return hipErrorOutOfMemory;
  const int64_t total = (nchunks - 1) * spc + last / kSeg;
  const int64_t waves = kThreads / 64;
  const int64_t cap = max_blocks > 0 ? max_blocks : 4 * 256;
  const unsigned grid = unsigned(std::min<int64_t>((total + waves - 1) / waves, cap));
  const auto* sp = static_cast<const uint8_t*>(src);
  switch (chains) {
    case 1:
      crc32c_mfma_segments_kernel<1><<<dim3(grid), dim3(kThreads), 0, s>>>(sp, bytes, chunk_bytes, spc, total, consts, sh,
                                                                           sh + spc * 32, seg_out);
      break;
    case 4:
      crc32c_mfma_segments_kernel<4><<<dim3(grid), dim3(kThreads), 0, s>>>(sp, bytes, chunk_bytes, spc, total, consts, sh,
                                                                           sh + spc * 32, seg_out);
      break;
    default:
      crc32c_mfma_segments_kernel<2><<<dim3(grid), dim3(kThreads), 0, s>>>(sp, bytes, chunk_bytes, spc, total, consts, sh,
                                                                           sh + spc * 32, seg_out);
  }
  return hipGetLastError();
}

}  // namespace kern
}  // namespace dissem
