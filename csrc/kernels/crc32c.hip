// Per-chunk CRC32C on gfx950 (receiver-side verification of every landed chunk).
//
// CRC is a serial recurrence, so the kernel works with raw (un-inverted) CRC
// registers, which are linear over GF(2):
//   raw(A || B) = shift(raw(A), |B|) xor raw(B),  shift(r, L) = r * x^(8L) mod P.
// Decomposition:
//  * a chunk is cut into 16 KiB segments; one wave owns a segment;
//  * lane l of the wave reads 16-B words l, l+64, l+128, ... (each wave
//    instruction reads 1 KiB contiguous: fully coalesced) and keeps the raw CRC
//    of its strided sub-message: s = shift_1KiB(s) xor crc16(word). Both maps
//    are GF(2)-linear, so one step is the XOR of 40 nibble-table lookups (32 for
//    the word's nibbles, 8 for the register's);
//  * each lane's CRC is shifted to the END OF ITS CHUNK with one GF(2)
//    multiply by a host-computed constant (per segment and lane: the lane's
//    distance to its segment end plus the segment's distance to the chunk
//    end), then the lanes are XOR-reduced with cross-lane shuffles, so
//  * a chunk's raw CRC is the plain XOR of its segments' values: a second,
//    small kernel XOR-reduces them (one 256-thread block per chunk) and adds
//    the init/xorout term, writing the standard CRC32C.
// The result is the exact CRC32C of each chunk for any chunk length that is a
// multiple of 16 (the buffer's final chunk may have any length).
//
// LDS layout (MI355X_MICROARCH.md, LDS): a ds_read_b32 is served in two groups
// of 32 lanes over 32 banks; with data-dependent indices a plain 256-entry table
// averages ~3 LDS cycles per group (bank conflicts measured at 2x the useful
// cycles in round 1, profiles/r1_counters). Each nibble table entry is stored
// 32 times, replica r in bank r, and lane l reads replica l & 31: conflict-free
// by construction (profiles/r1_crc_ab: SQ_LDS_BANK_CONFLICT = 0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "core/crc32c.h"
#include "kernels/kernels.h"

namespace dissem {
namespace kern {

namespace {

// 16 KiB per wave: 16 strided words per lane. One 64 MiB landing chunk spreads
// over 4096 waves (16 per CU).
constexpr int kSegBytes = 16 * 1024;
constexpr int kWordsPerLane = kSegBytes / 16 / 64;
constexpr int kNibTables = 40;  // 32 for a 16-B word, 8 for the register shifted by 1 KiB
// Global constants: [T0: 256][lanepow: 64][nibble tables: 40 x 16].
constexpr int kOffT0 = 0;
constexpr int kOffLanePow = 256;
constexpr int kOffNib = 256 + 64;
constexpr int kConstWords = kOffNib + kNibTables * 16;
// 40 tables x 16 entries x 32 replicas x 4 B = 80 KiB: two workgroups per CU.
constexpr int kNibLds = kNibTables * 16 * 32;

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

__device__ inline uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}

// XOR of the 8 nibble tables t0..t0+7, indexed by the 8 nibbles of x.
// L = lds + (lane & 31): entry (t, v) of this lane's bank-private replica.
__device__ __forceinline__ uint32_t nib8(const uint32_t* L, int t0, uint32_t x) {
  uint32_t r = 0;
#pragma unroll
  for (int n = 0; n < 8; ++n) r ^= L[(t0 + n) * 512 + ((x >> (4 * n)) & 15) * 32];
  return r;
}

// One strided step of a lane: s = shift_1KiB(s) xor crc16raw(w).
__device__ __forceinline__ uint32_t nib_step(const uint32_t* L, uint32_t s, uint4 w) {
  return nib8(L, 32, s) ^ nib8(L, 0, w.x) ^ nib8(L, 8, w.y) ^ nib8(L, 16, w.z) ^ nib8(L, 24, w.w);
}

__device__ inline void load_nib_lds(uint32_t* lds, const uint32_t* __restrict__ consts) {
  // 32 identical replicas per entry, written 4 at a time (16-B stores).
  const uint32_t* nib = consts + kOffNib;
  for (int i = threadIdx.x; i < kNibLds / 4; i += blockDim.x) {
    const uint32_t v = nib[i >> 3];
    reinterpret_cast<uint4*>(lds)[i] = make_uint4(v, v, v, v);
  }
  __syncthreads();
}

// One 16 KiB segment on one wave: the raw CRC of [seg, seg + seg_len), shifted
// to its chunk end (full segments: lane l multiplies by shift_row[l]; a partial
// segment is always its chunk's last, so its lanes only align to it). The
// result is valid in lane 0. Visit sees every 16-B word with its byte offset
// in the chunk (seg_start + offset in the segment).
struct NibStep {  // bank-private nibble tables (load_nib_lds layout)
  const uint32_t* L;
  __device__ __forceinline__ uint32_t operator()(uint32_t s, uint4 w) const { return nib_step(L, s, w); }
};

template <int DEPTH, class Visit, class Step>
__device__ __forceinline__ uint32_t one_segment_s(const uint8_t* __restrict__ seg, int64_t seg_start, int64_t seg_len,
                                         const uint32_t* __restrict__ shift_row,
                                         const uint32_t* __restrict__ consts, const Step& step, int lane,
                                         Visit& visit) {
  const int64_t nw = seg_len >> 4;
  const uint4* words = reinterpret_cast<const uint4*>(seg);
  uint32_t s = 0;
  if (nw == kSegBytes / 16) {
    // Full segment: 16 strided words per lane, DEPTH loads in flight per batch.
    using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int b = 0; b < kWordsPerLane; b += DEPTH) {
      u32x4 wv[DEPTH];
#pragma unroll
      for (int i = 0; i < DEPTH; ++i)
        wv[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(words + lane + 64 * (b + i)));
#pragma unroll
      for (int i = 0; i < DEPTH; ++i) {
        const uint4 w = make_uint4(wv[i][0], wv[i][1], wv[i][2], wv[i][3]);
        s = step(s, w);
        visit(w, seg_start + 16 * (lane + 64 * (b + i)));
      }
    }
    s = multmodp(shift_row[lane], s);
  } else {
    int64_t last = -1;
    for (int64_t j = lane; j < nw; j += 64) {
      const uint4 w = words[j];
      s = step(s, w);
      visit(w, seg_start + 16 * j);
      last = j;
    }
    if (last >= 0) s = multmodp(consts[kOffLanePow + nw - 1 - last], s);
  }
  s = wave_xor(s);
  if (lane == 0) {
    // Byte tail (only a buffer's final segment can have one).
    const uint8_t* tail = seg + (nw << 4);
    for (int64_t b = 0; b < (seg_len & 15); ++b) s = consts[kOffT0 + ((s ^ tail[b]) & 255)] ^ (s >> 8);
  }
  return s;
}

template <int DEPTH, class Visit>
__device__ __forceinline__ uint32_t one_segment(const uint8_t* __restrict__ seg, int64_t seg_start, int64_t seg_len,
                                       const uint32_t* __restrict__ shift_row,
                                       const uint32_t* __restrict__ consts, const uint32_t* L, int lane,
                                       Visit& visit) {
  return one_segment_s<DEPTH>(seg, seg_start, seg_len, shift_row, consts, NibStep{L}, lane, visit);
}

// ---- byte-addressed table layout (v2): fewer VALU per lookup ----
// A lookup address is (nibble << stride) | lane_offset + table offset. In the
// layout above every nibble is first shifted down and then scaled (2 VALU
// before the ds_read). Here a byte of the value is moved to bits 8-15 once (one
// shift per byte, none for byte 1) and both of its nibbles are masked in place:
// the low nibble (bits 8-11) indexes tables with 256-B entry stride (two tables
// interleaved per 4 KiB), the high nibble (bits 12-15) tables with 4-KiB stride
// (up to 32 interleaved, 128 B apart). Each entry still holds 32 replicas, one
// per bank, and lane l reads replica l & 31: conflict-free as before. Per
// 32-bit value: 3 shifts + 8 and-or + 8 xor instead of 16 + 8.
// Tables: 20 low-nibble (class A) and 20 high-nibble (class B) tables, index
// idx = byte position (data bytes 0-15, state bytes 16-19).
constexpr uint32_t kNib2B = 40960;                 // class A: 10 pairs x 4 KiB
constexpr uint32_t kNib2Bytes = kNib2B + 65536;    // class B: 16 rows x 4 KiB
constexpr int kSeg2Threads = 1024;                 // one 104 KiB workgroup per CU, 4 waves per SIMD

__device__ __forceinline__ uint32_t lds_word(const uint8_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(lds + byte_addr);
}

template <int IDX>  // v: the value with this byte at bits 8-15
__device__ __forceinline__ uint32_t byte_lookup2(const uint8_t* lds, uint32_t v, uint32_t lo) {
  constexpr uint32_t offA = (IDX >> 1) * 4096u + (IDX & 1) * 128u;
  constexpr uint32_t offB = kNib2B + IDX * 128u;
  return lds_word(lds, ((v & 0xF00u) | lo) + offA) ^ lds_word(lds, ((v & 0xF000u) | lo) + offB);
}

template <int K0>  // the 4 bytes of x are byte positions K0..K0+3
__device__ __forceinline__ uint32_t bytes4_lookup2(const uint8_t* lds, uint32_t x, uint32_t lo) {
  return byte_lookup2<K0>(lds, x << 8, lo) ^ byte_lookup2<K0 + 1>(lds, x, lo) ^
         byte_lookup2<K0 + 2>(lds, x >> 8, lo) ^ byte_lookup2<K0 + 3>(lds, x >> 16, lo);
}

struct NibStep2 {
  const uint8_t* lds;
  uint32_t lo;  // (lane & 31) * 4: this lane's replica
  __device__ __forceinline__ uint32_t operator()(uint32_t s, uint4 w) const {
    return bytes4_lookup2<16>(lds, s, lo) ^ bytes4_lookup2<0>(lds, w.x, lo) ^ bytes4_lookup2<4>(lds, w.y, lo) ^
           bytes4_lookup2<8>(lds, w.z, lo) ^ bytes4_lookup2<12>(lds, w.w, lo);
  }
};

__device__ inline void load_nib2_lds(uint8_t* lds, const uint32_t* __restrict__ consts) {
  // same 40 x 16 table values as load_nib_lds (t = 2 * byte + hi), 32 replicas as 8 x 16 B
  const uint32_t* nib = consts + kOffNib;
  for (int i = threadIdx.x; i < kNibTables * 16 * 8; i += blockDim.x) {
    const int e = i >> 3, q = i & 7;
    const int t = e >> 4, v = e & 15, idx = t >> 1;
    const uint32_t val = nib[e];
    const uint32_t addr = (t & 1) ? kNib2B + uint32_t(v) * 4096u + uint32_t(idx) * 128u
                                  : uint32_t(idx >> 1) * 4096u + uint32_t(v) * 256u + uint32_t(idx & 1) * 128u;
    reinterpret_cast<uint4*>(lds + addr)[q] = make_uint4(val, val, val, val);
  }
  __syncthreads();
}

// Segment walk of the plain and the fused kernels: `bytes` cut into chunks of
// `chunk_bytes`, each wave owns 16 KiB segments (grid-stride). seg_out[g] gets
// the segment's raw CRC shifted to the end of its chunk (shift: lane
// constants of full chunks, shift_last: of a shorter final chunk).
template <int DEPTH, class Visit>
__device__ __forceinline__ void segment_crcs(const uint8_t* __restrict__ src, int64_t bytes, int64_t chunk_bytes,
                                    int64_t spc, int64_t total_segs, const uint32_t* __restrict__ consts,
                                    const uint32_t* __restrict__ shift, const uint32_t* __restrict__ shift_last,
                                    uint32_t* __restrict__ seg_out, const uint32_t* lds, Visit& visit) {
  const int lane = threadIdx.x & 63;
  const uint32_t* L = lds + (lane & 31);
  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x / 64);
  for (int64_t g = wave; g < total_segs; g += nwaves) {
    const int64_t c = g / spc, k = g % spc;
    const int64_t chunk_start = c * chunk_bytes;
    const int64_t chunk_len = min(chunk_bytes, bytes - chunk_start);
    const int64_t seg_start = k * kSegBytes;
    const int64_t seg_len = min(int64_t(kSegBytes), chunk_len - seg_start);
    visit.begin(c, chunk_start, chunk_len);
    const uint32_t* row = (chunk_len == chunk_bytes ? shift : shift_last) + k * 64;
    const uint32_t s = one_segment<DEPTH>(src + chunk_start + seg_start, seg_start, seg_len, row, consts, L, lane,
                                          visit);
    if (lane == 0) seg_out[g] = s;
  }
}

struct NoVisit {
  __device__ void begin(int64_t, int64_t, int64_t) {}
  __device__ void operator()(const uint4&, int64_t) {}
};

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
// [q: n bytes][scales: n/BLOCK f32] per chunk): while computing each segment's
// CRC, words in the q region are dequantized and written as bf16. Every packed
// byte is read once from HBM; the scales (1/32 of the traffic) come from L2.
template <int BLOCK>
struct UnpackVisit {
  int64_t out_chunk_elems;
  uint16_t* out;
  const uint8_t* src;
  int64_t n_q = 0;
  const float* scales = nullptr;
  uint16_t* obase = nullptr;
  __device__ void begin(int64_t c, int64_t chunk_start, int64_t chunk_len) {
    n_q = chunk_len / (BLOCK + 4) * BLOCK;  // q bytes (= elements) of this chunk
    scales = reinterpret_cast<const float*>(src + chunk_start + n_q);
    obase = out + c * out_chunk_elems;
  }
  __device__ void operator()(const uint4& w, int64_t e) {  // e: byte offset in chunk = element index in q
    if (e < n_q) unpack16(w, scales[e / BLOCK], reinterpret_cast<uint4*>(obase + e));
  }
};

// Launch shape: 512 threads (8 waves), two workgroups per CU (LDS-bound at
// 80 KiB each); waves_per_eu(4) keeps VGPRs <= 128 so both fit.
constexpr int kSegThreads = 512;

__global__ void __launch_bounds__(kSegThreads) __attribute__((amdgpu_waves_per_eu(4)))
crc32c_segments_kernel(const uint8_t* __restrict__ src, int64_t bytes, int64_t chunk_bytes, int64_t spc,
                       int64_t total_segs, const uint32_t* __restrict__ consts, const uint32_t* __restrict__ shift,
                       const uint32_t* __restrict__ shift_last, uint32_t* __restrict__ seg_out) {
  __shared__ uint32_t lds[kNibLds];
  load_nib_lds(lds, consts);
  NoVisit v;
  segment_crcs<16>(src, bytes, chunk_bytes, spc, total_segs, consts, shift, shift_last, seg_out, lds, v);
}

// Rolling prefetch: a wave that owns several full segments issues the load of
// word i of its NEXT segment right after consuming word i of the current one,
// so the next segment's 16 KiB is in flight while this one's lookups run (the
// same 64 data VGPRs as the plain kernel). The segment index math is
// wave-uniform (scalar). Partial segments take the plain path.
template <class Step>
__device__ __forceinline__ void roll_walk(const uint8_t* __restrict__ src, int64_t bytes, int64_t chunk_bytes,
                                          int64_t spc, int64_t total_segs, const uint32_t* __restrict__ consts,
                                          const uint32_t* __restrict__ shift, const uint32_t* __restrict__ shift_last,
                                          uint32_t* __restrict__ seg_out, const Step& step) {
  using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int64_t wave =
      __builtin_amdgcn_readfirstlane(int(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)));
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x / 64);
  struct Geo {
    int64_t chunk_start, chunk_len, seg_start, seg_len, k;
  };
  auto geo = [&](int64_t g) {
    Geo o;
    const int64_t c = g / spc;
    o.k = g - c * spc;
    o.chunk_start = c * chunk_bytes;
    o.chunk_len = min(chunk_bytes, bytes - o.chunk_start);
    o.seg_start = o.k * kSegBytes;
    o.seg_len = min(int64_t(kSegBytes), o.chunk_len - o.seg_start);
    return o;
  };
  u32x4 w[kWordsPerLane];
  bool loaded = false;
  NoVisit v;
  int64_t g = wave;
  if (g >= total_segs) return;
  Geo cur = geo(g);
  for (; g < total_segs; g += nwaves) {
    const u32x4* cw = reinterpret_cast<const u32x4*>(src + cur.chunk_start + cur.seg_start);
    const int64_t gn = g + nwaves;
    Geo nxt{};
    bool nfull = false;
    if (gn < total_segs) {
      nxt = geo(gn);
      nfull = nxt.seg_len == kSegBytes;
    }
    const uint32_t* row = (cur.chunk_len == chunk_bytes ? shift : shift_last) + cur.k * 64;
    uint32_t s;
    if (cur.seg_len == kSegBytes) {
      if (!loaded) {
#pragma unroll
        for (int i = 0; i < kWordsPerLane; ++i) w[i] = __builtin_nontemporal_load(cw + lane + 64 * i);
      }
      // no next full segment: the prefetch re-reads this one (harmless, in bounds)
      const u32x4* nw = nfull ? reinterpret_cast<const u32x4*>(src + nxt.chunk_start + nxt.seg_start) : cw;
      s = 0;
#pragma unroll
      for (int i = 0; i < kWordsPerLane; ++i) {
        const u32x4 x = w[i];
        w[i] = __builtin_nontemporal_load(nw + lane + 64 * i);
        s = step(s, make_uint4(x[0], x[1], x[2], x[3]));
      }
      loaded = nfull;
      s = wave_xor(multmodp(row[lane], s));
    } else {
      s = one_segment_s<4>(src + cur.chunk_start + cur.seg_start, cur.seg_start, cur.seg_len, row, consts, step, lane,
                           v);
      loaded = false;
    }
    if (lane == 0) seg_out[g] = s;
    cur = nxt;
  }
}

// Byte-addressed tables (v2 layout above) + rolling prefetch.
__global__ void __launch_bounds__(kSeg2Threads) __attribute__((amdgpu_waves_per_eu(4)))
crc32c_segments_roll2_kernel(const uint8_t* __restrict__ src, int64_t bytes, int64_t chunk_bytes, int64_t spc,
                             int64_t total_segs, const uint32_t* __restrict__ consts,
                             const uint32_t* __restrict__ shift, const uint32_t* __restrict__ shift_last,
                             uint32_t* __restrict__ seg_out) {
  __shared__ uint4 lds[kNib2Bytes / 16];
  uint8_t* base = reinterpret_cast<uint8_t*>(lds);
  load_nib2_lds(base, consts);
  roll_walk(src, bytes, chunk_bytes, spc, total_segs, consts, shift, shift_last, seg_out,
            NibStep2{base, (threadIdx.x & 31u) * 4u});
}

template <int BLOCK>
__global__ void __launch_bounds__(kSegThreads) __attribute__((amdgpu_waves_per_eu(4)))
verify_unpack_segments_kernel(const uint8_t* __restrict__ src, int64_t bytes, int64_t pchunk, int64_t spc,
                              int64_t total_segs, int64_t out_chunk_elems, const uint32_t* __restrict__ consts,
                              const uint32_t* __restrict__ shift, const uint32_t* __restrict__ shift_last,
                              uint32_t* __restrict__ seg_out, uint16_t* __restrict__ out) {
  __shared__ uint32_t lds[kNibLds];
  load_nib_lds(lds, consts);
  UnpackVisit<BLOCK> v{out_chunk_elems, out, src};
  segment_crcs<4>(src, bytes, pchunk, spc, total_segs, consts, shift, shift_last, seg_out, lds, v);
}

// One 256-thread block per chunk: XOR of the chunk's (pre-shifted) segment
// values plus the init/xorout term. init[0]: full chunks, init[1]: short last chunk.
__global__ void __launch_bounds__(256) crc32c_fold_kernel(const uint32_t* __restrict__ seg_out, int64_t bytes,
                                                          int64_t chunk_bytes, int64_t spc,
                                                          const uint32_t* __restrict__ init,
                                                          uint32_t* __restrict__ out) {
  __shared__ uint32_t part[4];
  const int64_t c = blockIdx.x;
  const int64_t chunk_len = min(chunk_bytes, bytes - c * chunk_bytes);
  const int64_t n = (chunk_len + kSegBytes - 1) / kSegBytes;
  const uint32_t* seg = seg_out + c * spc;
  uint32_t r = 0;
  for (int64_t k = threadIdx.x; k < n; k += 256) r ^= seg[k];
  r = wave_xor(r);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = r;
  __syncthreads();
  if (threadIdx.x == 0) out[c] = part[0] ^ part[1] ^ part[2] ^ part[3] ^ init[chunk_len == chunk_bytes ? 0 : 1];
}

// ---- batched: up to kCrcBatchMax independent buffers (the chunks one P2P
// group landed) in one segments launch + one fold launch.
struct BatchArgs {
  int n;
  int64_t seg_base[kCrcBatchMax + 1];  // prefix sums of the items' segment counts
  const uint8_t* src[kCrcBatchMax];
  int64_t bytes[kCrcBatchMax];
  const uint32_t* shift[kCrcBatchMax];  // lane shift table of a `bytes`-byte chunk
  uint32_t init[kCrcBatchMax];
  uint32_t* out[kCrcBatchMax];
};

__global__ void __launch_bounds__(kSegThreads) __attribute__((amdgpu_waves_per_eu(4)))
crc32c_batch_segments_kernel(const BatchArgs a, const uint32_t* __restrict__ consts, uint32_t* __restrict__ seg_out) {
  __shared__ uint32_t lds[kNibLds];
  load_nib_lds(lds, consts);
  const int lane = threadIdx.x & 63;
  const uint32_t* L = lds + (lane & 31);
  const int64_t wave = int64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x / 64);
  NoVisit v;
  for (int64_t g = wave; g < a.seg_base[a.n]; g += nwaves) {
    int j = 0;
    while (g >= a.seg_base[j + 1]) ++j;
    const int64_t k = g - a.seg_base[j];
    const int64_t seg_start = k * kSegBytes;
    const int64_t seg_len = min(int64_t(kSegBytes), a.bytes[j] - seg_start);
    const uint32_t s = one_segment<16>(a.src[j] + seg_start, seg_start, seg_len, a.shift[j] + k * 64, consts, L,
                                       lane, v);
    if (lane == 0) seg_out[g] = s;
  }
}

__global__ void __launch_bounds__(256) crc32c_batch_fold_kernel(const BatchArgs a,
                                                                const uint32_t* __restrict__ seg_out) {
  __shared__ uint32_t part[4];
  const int j = blockIdx.x;
  uint32_t r = 0;
  for (int64_t g = a.seg_base[j] + threadIdx.x; g < a.seg_base[j + 1]; g += 256) r ^= seg_out[g];
  r = wave_xor(r);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = r;
  __syncthreads();
  if (threadIdx.x == 0) *a.out[j] = part[0] ^ part[1] ^ part[2] ^ part[3] ^ a.init[j];
}

// Per-device constant tables and per-(chunk, last chunk) fold tables.
struct DeviceConsts {
  std::mutex mu;
  std::map<int, uint32_t*> by_device;
  // (device, chunk_bytes, last_len) -> [shift: spc x 64][shift_last: spc x 64][init: 2]
  std::map<std::tuple<int, int64_t, int64_t>, uint32_t*> fold;
};
DeviceConsts g_consts;

// Per full segment k of a `len`-byte chunk and lane l: x^(8 * (bytes from the
// end of lane l's last word to the chunk end)) = x^(8*16*(63 - l)) * x^(8 * (len - end of k)).
void lane_shifts(int64_t len, int64_t spc, uint32_t* out) {
  const int64_t nfull = len / kSegBytes;
  std::fill(out, out + spc * 64, 0u);  // partial / absent segments: unused
  if (nfull == 0) return;
  uint32_t lanepow[64];
  for (int m = 0; m < 64; ++m) lanepow[m] = crc32c_xpow8n(uint64_t(16) * uint64_t(m));
  const uint32_t xs = crc32c_xpow8n(kSegBytes);
  uint32_t seg = crc32c_xpow8n(uint64_t(len - nfull * kSegBytes));  // last full segment
  for (int64_t k = nfull - 1; k >= 0; --k) {
    for (int l = 0; l < 64; ++l) out[k * 64 + l] = crc32c_multmodp(lanepow[63 - l], seg);
    seg = crc32c_multmodp(xs, seg);
  }
}

uint32_t* fold_consts(int64_t chunk_bytes, int64_t last_len) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_consts.mu);
  auto key = std::make_tuple(dev, chunk_bytes, last_len);
  auto it = g_consts.fold.find(key);
  if (it != g_consts.fold.end()) return it->second;
  const int64_t spc = (chunk_bytes + kSegBytes - 1) / kSegBytes;
  std::vector<uint32_t> h(size_t(2 * spc * 64 + 2));
  lane_shifts(chunk_bytes, spc, h.data());
  lane_shifts(last_len, spc, h.data() + spc * 64);
  h[size_t(2 * spc * 64)] = crc32c_init_term(uint64_t(chunk_bytes));
  h[size_t(2 * spc * 64 + 1)] = crc32c_init_term(uint64_t(last_len));
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
  std::vector<uint32_t> T(16 * 256), A(4 * 256), h(kConstWords);
  crc32c_slice16_tables(T.data());
  crc32c_shift_tables(1024, A.data());
  for (int i = 0; i < 256; ++i) h[size_t(kOffT0 + i)] = T[size_t(i)];
  for (int m = 0; m < 64; ++m) h[size_t(kOffLanePow + m)] = crc32c_xpow8n(uint64_t(16) * uint64_t(m));
  // Nibble tables: t = 2k + hi for data byte k (slice-by-16 table 15 - k),
  // t = 32 + 2i + hi for byte i of the register (1 KiB shift map).
  for (int t = 0; t < kNibTables; ++t)
    for (uint32_t v = 0; v < 16; ++v) {
      const uint32_t byte = v << (4 * (t & 1));
      h[size_t(kOffNib + t * 16 + int(v))] =
          t < 32 ? T[size_t((15 - t / 2) * 256) + byte] : A[size_t(((t - 32) / 2) * 256) + byte];
    }
  uint32_t* d = nullptr;
  if (hipMalloc(&d, h.size() * 4) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  g_consts.by_device[dev] = d;
  return d;
}

// Two workgroups per CU, one 16 KiB segment per wave (grid-stride beyond that).
dim3 seg_grid(int64_t total_segs) {
  const int64_t waves = kSegThreads / 64;
  return dim3(unsigned(std::min<int64_t>((total_segs + waves - 1) / waves, 2 * 256)));
}

struct Plan {
  int64_t spc, nchunks, total_segs;
  uint32_t *consts, *fold;
};

hipError_t plan(int64_t bytes, int64_t chunk_bytes, Plan* p) {
  p->spc = (chunk_bytes + kSegBytes - 1) / kSegBytes;
  p->nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  const int64_t last_len = bytes - (p->nchunks - 1) * chunk_bytes;
  p->total_segs = (p->nchunks - 1) * p->spc + (last_len + kSegBytes - 1) / kSegBytes;
  p->consts = device_consts();
  p->fold = fold_consts(chunk_bytes, last_len);
  return p->consts && p->fold ? hipSuccess : hipErrorOutOfMemory;
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
  return crc32c_chunks_impl(src, bytes, chunk_bytes, out, workspace, s, CrcImpl::kAuto, 0);
}

hipError_t crc32c_chunks_impl(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                              hipStream_t s, CrcImpl impl, int max_blocks) {
  if (bytes <= 0) return hipSuccess;
  if (chunk_bytes <= 0 || chunk_bytes % 16 || (reinterpret_cast<uintptr_t>(src) & 15)) return hipErrorInvalidValue;
  Plan p;
  if (hipError_t e = plan(bytes, chunk_bytes, &p); e != hipSuccess) return e;
  auto* seg = static_cast<uint32_t*>(workspace);
  if (impl == CrcImpl::kRolling ||
      (impl == CrcImpl::kAuto && p.total_segs >= 2 * int64_t(256) * (kSeg2Threads / 64))) {
    // bulk launches where every wave of the full grid owns >= 2 segments:
    // 3.32 TB/s on 1 GiB vs 2.69 for the plain kernel; a single 64 MiB chunk
    // has one segment per wave - nothing to overlap - and stays on the plain
    // kernel: 31 vs 38 us (profiles/r2_crc_ab/crc_roll2.json)
    const int64_t waves = kSeg2Threads / 64;
    const int64_t cap = max_blocks > 0 ? max_blocks : 256;
    const dim3 grid(unsigned(std::max<int64_t>(1, std::min<int64_t>((p.total_segs + waves - 1) / waves, cap))));
    crc32c_segments_roll2_kernel<<<grid, dim3(kSeg2Threads), 0, s>>>(
        static_cast<const uint8_t*>(src), bytes, chunk_bytes, p.spc, p.total_segs, p.consts, p.fold,
        p.fold + p.spc * 64, seg);
  } else {
    crc32c_segments_kernel<<<seg_grid(p.total_segs), dim3(kSegThreads), 0, s>>>(
        static_cast<const uint8_t*>(src), bytes, chunk_bytes, p.spc, p.total_segs, p.consts, p.fold,
        p.fold + p.spc * 64, seg);
  }
  crc32c_fold_kernel<<<dim3(unsigned(p.nchunks)), dim3(256), 0, s>>>(seg, bytes, chunk_bytes, p.spc,
                                                                     p.fold + 2 * p.spc * 64, out);
  return hipGetLastError();
}

size_t crc32c_batch_workspace_bytes(int64_t max_item_bytes, int n) {
  const int64_t spc = (std::max<int64_t>(max_item_bytes, 1) + kSegBytes - 1) / kSegBytes;
  return size_t(int64_t(std::max(n, 1)) * spc * 4 + 16);
}

hipError_t crc32c_batch(const CrcItem* items, int n, void* workspace, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n > kCrcBatchMax) return hipErrorInvalidValue;
  BatchArgs a{};
  a.n = 0;
  a.seg_base[0] = 0;
  uint32_t* consts = device_consts();
  if (!consts) return hipErrorOutOfMemory;
  for (int i = 0; i < n; ++i) {
    const CrcItem& it = items[i];
    if (it.bytes <= 0) continue;
    if (it.bytes % 16 || (reinterpret_cast<uintptr_t>(it.src) & 15)) return hipErrorInvalidValue;
    uint32_t* fold = fold_consts(it.bytes, it.bytes);
    if (!fold) return hipErrorOutOfMemory;
    const int64_t spc = (it.bytes + kSegBytes - 1) / kSegBytes;
    const int j = a.n++;
    a.src[j] = static_cast<const uint8_t*>(it.src);
    a.bytes[j] = it.bytes;
    a.shift[j] = fold;
    a.init[j] = crc32c_init_term(uint64_t(it.bytes));
    a.out[j] = it.out;
    a.seg_base[j + 1] = a.seg_base[j] + spc;
  }
  if (a.n == 0) return hipSuccess;
  auto* seg = static_cast<uint32_t*>(workspace);
  crc32c_batch_segments_kernel<<<seg_grid(a.seg_base[a.n]), dim3(kSegThreads), 0, s>>>(a, consts, seg);
  crc32c_batch_fold_kernel<<<dim3(unsigned(a.n)), dim3(256), 0, s>>>(a, seg);
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
  Plan p;
  if (hipError_t e = plan(bytes, pchunk, &p); e != hipSuccess) return e;
  auto* seg = static_cast<uint32_t*>(workspace);
  auto* src = static_cast<const uint8_t*>(packed);
  const int64_t oc = src_chunk / 2;
  const dim3 grid = seg_grid(p.total_segs), tpb{kSegThreads};
  const uint32_t *sp = p.fold, *sl = p.fold + p.spc * 64;
  switch (block) {
    case 32: verify_unpack_segments_kernel<32><<<grid, tpb, 0, s>>>(src, bytes, pchunk, p.spc, p.total_segs, oc, p.consts, sp, sl, seg, out); break;
    case 64: verify_unpack_segments_kernel<64><<<grid, tpb, 0, s>>>(src, bytes, pchunk, p.spc, p.total_segs, oc, p.consts, sp, sl, seg, out); break;
    case 128: verify_unpack_segments_kernel<128><<<grid, tpb, 0, s>>>(src, bytes, pchunk, p.spc, p.total_segs, oc, p.consts, sp, sl, seg, out); break;
    case 256: verify_unpack_segments_kernel<256><<<grid, tpb, 0, s>>>(src, bytes, pchunk, p.spc, p.total_segs, oc, p.consts, sp, sl, seg, out); break;
    case 512: verify_unpack_segments_kernel<512><<<grid, tpb, 0, s>>>(src, bytes, pchunk, p.spc, p.total_segs, oc, p.consts, sp, sl, seg, out); break;
    default: return hipErrorInvalidValue;
  }
  crc32c_fold_kernel<<<dim3(unsigned(p.nchunks)), dim3(256), 0, s>>>(seg, bytes, pchunk, p.spc,
                                                                     p.fold + 2 * p.spc * 64, crc_out);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace dissem
