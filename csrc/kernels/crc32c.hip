// CRC32C on gfx950 (receiver-side verification of every landed chunk), and
// the fused CRC32C + fp8 -> bf16 dequantization of packed chunks.
//
// CRC is a serial recurrence, so the kernel works with raw (un-inverted) CRC
// registers, which are linear over GF(2):
//   raw(A || B) = shift(raw(A), |B|) xor raw(B),  shift(r, L) = r * x^(8L) mod P.
// Decomposition:
//  * a chunk is cut into 16 KiB segments; one wave owns a segment at a time
//    (the fused kernel: one segment per wave, the last, partial round of its
//    grid half a segment, see once_split; the CRC-only kernel: a walk over a
//    per-workgroup range of segments);
//  * a segment is 4 blocks of 4 KiB, and lane l owns the contiguous 64-B piece
//    l of every block. Within a piece the classic slice-by-4 recurrence runs
//    (s ^= word; s = T3[b0] ^ T2[b1] ^ T1[b2] ^ T0[b3]): one table lookup per
//    byte. Between its pieces a lane's register crosses the 4032 bytes of the
//    other lanes as zeros: a fixed GF(2)-linear map, 8 nibble lookups;
//  * each lane's CRC is shifted to the END OF ITS SEGMENT with one GF(2)
//    multiply by a per-lane constant (x^(8*64*(63-lane))), then the lanes are
//    XOR-reduced with cross-lane shuffles: a segment's value is its raw CRC
//    (the walk does this once per run of a wave's segments of one chunk,
//    carrying each lane's register across the segments between: crc_walk);
//  * the wave then shifts that value to the END OF ITS CHUNK - x^(8*16 KiB*j)
//    from three 1024-entry levels of a table, then x^(8*rem) for a chunk whose
//    last segment is short (wave-uniform products);
//  * the fold runs in the same launch: a workgroup XORs its waves' values per
//    chunk (in LDS) and adds them to the chunk's {acc, count} word with
//    device-scope atomics; the workgroup that completes the count writes the standard
//    CRC32C (fold_add below). The separate fold launch this replaced cost
//    8.4-9.6 us per 64 MiB chunk in the round-4 engine traces.
// One launch covers a regular chunk grid (ChunkGeo) or up to kCrcBatchMax
// independent chunks (BatchGeo: the chunks one P2P issue pass or one staging
// batch landed). The constants depend on nothing but the segment geometry
// (chunks up to 16 TiB): one upload per device, never a per-length table.
// The result is the exact CRC32C of each chunk for any chunk length that is a
// multiple of 16 (a buffer's final chunk, and a batch item, may have any length).
//
// Loads stay coalesced: each 16-B load instruction of a wave reads one whole
// KiB (lane m + 16 r: word r of piece 16 j + m of KiB j), and a 4x4 register
// transpose across the wave's 4 rows (v_permlane16_swap / v_permlane32_swap,
// 16 VALU per 64 B of lane data) hands lane l its piece l. Loading the pieces
// directly (every lane 16 B of its own piece per instruction: 64 separate
// 64-B spans) reads at 3.5-4.0 TB/s against 6.8 for whole KiBs in the same
// 16-KiB-per-wave shape (round 2's read-shape probe kernel, profiles/r2_crc_ab).
//
// LDS layout (MI355X_MICROARCH.md, LDS): a ds_read_b32 is served in two groups
// of 32 lanes over 32 banks, and data-dependent indices into a plain table
// conflict (2x the useful LDS cycles in round 1, profiles/r1_counters). Every
// table entry is stored R times, replica r in bank r, and lane l reads replica
// l mod R: R = 32 is conflict-free by construction (144 KiB: one workgroup
// per CU, the CRC-only walk); the fused kernel uses R = 16 in 72 KiB, so two
// 512-thread workgroups share a CU and one fills its tables and waits for its
// first loads while the other computes. Lanes l and l + 16 then share a
// replica, so each 16-lane group reads a different table in one instruction
// (Slice4T: lookup k on byte k ^ group; LdsLayout<16>::gap_entry) - as
// conflict-free as R = 32 (2.5e6 vs 2.95e7 conflict cycles, profiles/r6_pmc2).
// The address of byte k of s is ONE v_perm_b32 of s with a per-lane constant,
// then the ds_read_b32.
//
// History (profiles/r2_crc_ab, r4_*): nibble tables on strided 16-B words (40
// lookups per 16 B; 2.7 TB/s on 1 GiB), the same on byte-addressed nibble
// tables with a rolling prefetch (3.3 TB/s), an MFMA GF(2) product (2.3 TB/s),
// slice-by-4 on directly loaded pieces (3.1 TB/s) and with 4 independent
// recurrences per lane (2.3-2.5 TB/s) all lost to the slice-by-4-on-pieces
// scheme above: 5.76 TB/s on 1 GiB as a persistent walk (round 2). Round 4's
// fused kernel found one segment per wave faster than any persistent walk for
// read+write (vmcnt counts loads and stores in order: a walking wave's next
// loads wait behind its stores; bin/walkprobe, profiles/r4_walk*), and two
// recurrences per lane or four chains per block measured the same as one
// chain: the cost a launch pays over the copy is its first and last waves'
// ~600 VALU + 256 LDS lookups per lane per segment with nothing to hide
// behind. Round 5 removed the separate fold kernels and the store variants
// from the library, batches the engine's chunks per launch, and keeps the walk
// (tables filled once per CU, no stores) for the CRC-only check only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <cstring>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <vector>

#include "core/crc32c.h"
#include "kernels/fp8_cvt.h"
#include "kernels/kernels.h"

namespace dissem {
namespace kern {

namespace {

constexpr int kSegBytes = 16 * 1024;
constexpr int kPieceBytes = 64;                         // a lane's contiguous piece of a block
constexpr int kBlockBytes = 64 * kPieceBytes;           // 4 KiB
constexpr int kBlocksPerSeg = kSegBytes / kBlockBytes;  // 4
constexpr int kGapBytes = kBlockBytes - kPieceBytes;    // between a lane's pieces
constexpr int kWaves16 = 8;    // waves per workgroup of the fused kernel (512 threads, 16 table replicas)
constexpr int kWalkWaves = 16;  // ... of the CRC walk (1024 threads, 32 replicas)
constexpr uint32_t kShLds = 131072;                     // shift tables after the byte tables
constexpr uint32_t kLdsBytes = kShLds + 8 * 16 * 128;   // 144 KiB
// Global constants: [T: 4 x 256 (T[k][v]: byte v then k zero bytes)]
// [gap: 8 x 16 nibble tables of the kGapBytes shift][pow16: 1024 (x^(8*16 m))]
// [lanepow: 64 (x^(8*64*(63-l)): lane l's last piece to its segment end)]
// [segpow: 3 levels x 1024 (x^(8*16 KiB*i*1024^L)): x^(8*16 KiB*j) for any j
// below 2^30 is the product of at most three entries - chunks up to 16 TiB
// (one 1 GiB-chunk table capped a single CRC at 1 GiB in round 4)]
// [walkgap: 8 x 16 nibble tables of the walk's shift from a lane's last piece
// of one segment to its first piece of the segment 16 later (crc_walk)].
constexpr int kSegLevels = 3, kSegLevel = 1024;
constexpr int64_t kMaxSegs = int64_t(1) << (10 * kSegLevels);
constexpr int kT = 0, kGap = 1024, kPow = kGap + 128, kLanePow = kPow + 1024, kSegPow = kLanePow + 64,
              kWalkGap = kSegPow + kSegLevels * kSegLevel, kConstWords = kWalkGap + 128;

using u32x4_t = unsigned int __attribute__((ext_vector_type(4)));

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

// a(x) * b(x) mod P with no branches: 32 unrolled steps, each a masked XOR and
// a conditional reduction (the loop above diverges per lane and costs ~3x the
// instructions; it stays for the rare partial segments).
__device__ __forceinline__ uint32_t multmodp_unrolled(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; --i) {
    p ^= b & (0u - ((a >> i) & 1u));
    b = (b >> 1) ^ (kCrc32cPoly & (0u - (b & 1u)));
  }
  return p;
}

__device__ inline uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}

// XOR of v over the wave, wave-uniform: DPP within each row of 16 lanes
// (quad swaps, half-row and row mirrors), then the 4 row results by readlane.
__device__ __forceinline__ uint32_t wave_xor_dpp(uint32_t v) {
  v ^= uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v ^= uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v ^= uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
  v ^= uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x140, 0xF, 0xF, false));  // row_mirror
  return uint32_t(__builtin_amdgcn_readlane(int(v), 0)) ^ uint32_t(__builtin_amdgcn_readlane(int(v), 16)) ^
         uint32_t(__builtin_amdgcn_readlane(int(v), 32)) ^ uint32_t(__builtin_amdgcn_readlane(int(v), 48));
}

__device__ __forceinline__ uint32_t lds_word(const uint8_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(lds + byte_addr);
}

// Table replicas per entry: 32 (one per bank of a ds_read_b32 lane group:
// conflict-free, 144 KiB with the shift tables, one workgroup per CU) or 16
// (lanes l and l + 16 share a bank: up to 2-way conflicts, 72 KiB, two
// workgroups per CU).
template <int R>
struct LdsLayout {
  static_assert(R == 32 || R == 16, "32 or 16 table replicas");
  static constexpr uint32_t kSh = R == 32 ? 131072u : 65536u;  // shift tables after the byte tables
  static constexpr uint32_t kBytes = kSh + 8u * 16u * uint32_t(R) * 4u;
  // shift table n, entry v (replica 0). R = 32: one entry after another (each
  // entry's 32 replicas fill the 32 banks). R = 16: tables 2k and 2k + 1
  // interleave per entry, so table n's replicas sit in banks 16 (n & 1) + r
  // whatever the entry - lanes l and l + 16 then read different banks when they
  // look up tables of different parity (Slice4T::gap).
  static __device__ __host__ constexpr uint32_t gap_entry(int n, int v) {
    return R == 32 ? uint32_t(n * 16 + v) * 128u
                   : uint32_t(n >> 1) * 2048u + uint32_t(v) * 128u + uint32_t(n & 1) * 64u;
  }
  // byte table t, entry b, replica r
  static __device__ __forceinline__ uint32_t entry(int t, int b) {
    return R == 32 ? uint32_t(t >> 1) * 65536u + uint32_t(b) * 256u + uint32_t(t & 1) * 128u
                   : uint32_t(b) * 256u + uint32_t(t) * 64u;
  }
};
static_assert(LdsLayout<32>::kBytes == kLdsBytes, "144 KiB layout");

// The fused kernel's fill: one entry per iteration. Its table reads queue
// behind the segment loads already in flight (one in-order vmcnt), and the
// CU's other workgroup computes meanwhile; holding more table words in
// registers here spilled its 128 VGPRs (load_lds below is the walk's).
template <int R>
__device__ inline void load_lds_strided(uint8_t* lds, const uint32_t* __restrict__ sc) {
  constexpr int Q = R / 4;  // 16-B stores per entry
  for (int i = threadIdx.x; i < 4 * 256 * Q; i += blockDim.x) {
    const int e = i / Q, q = i % Q, t = e >> 8, b = e & 255;
    const uint32_t v = sc[kT + e];
    reinterpret_cast<uint4*>(lds + LdsLayout<R>::entry(t, b))[q] = make_uint4(v, v, v, v);
  }
  for (int i = threadIdx.x; i < 8 * 16 * Q; i += blockDim.x) {
    const int e = i / Q, q = i % Q;
    const uint32_t v = sc[kGap + e];
    reinterpret_cast<uint4*>(lds + LdsLayout<R>::kSh + LdsLayout<R>::gap_entry(e >> 4, e & 15))[q] =
        make_uint4(v, v, v, v);
  }
  __syncthreads();
}

// The walk's fill by its NT threads: each thread issues all of its table
// reads together, then writes its 16-B units in address order (consecutive
// lanes, consecutive units: conflict-free) - one global round trip per
// workgroup, where the strided loop above waits one per iteration (8) before
// the walk's first lookup. `walk_gap` (bytes; 0 = none): also copy the 128
// walk_gap words there.
template <int R, int NT>
__device__ __forceinline__ void load_lds(uint8_t* lds, const uint32_t* __restrict__ sc, uint32_t walk_gap = 0) {
  constexpr int kUnits = 4 * 256 * R / 4, kGapUnits = 8 * 16 * R / 4, K = kUnits / NT;
  static_assert(kUnits % NT == 0 && kGapUnits <= NT && 128 <= NT, "fill shape");
  static_assert(R == 32, "shift tables written in entry order (LdsLayout<32>::gap_entry)");
  const int tid = threadIdx.x;
  uint32_t v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t u = uint32_t(tid + k * NT);  // unit -> (table, byte) of LdsLayout<R>::entry
    const uint32_t t = R == 32 ? ((u >> 12) << 1) | ((u >> 3) & 1u) : (u >> 2) & 3u;
    const uint32_t b = R == 32 ? (u >> 4) & 255u : u >> 4;
    v[k] = sc[kT + t * 256u + b];
  }
  const uint32_t gv = tid < kGapUnits ? sc[kGap + tid / (R / 4)] : 0u;
  const uint32_t wv = walk_gap && tid < 128 ? sc[kWalkGap + tid] : 0u;
#pragma unroll
  for (int k = 0; k < K; ++k) reinterpret_cast<uint4*>(lds)[tid + k * NT] = make_uint4(v[k], v[k], v[k], v[k]);
  if (tid < kGapUnits) reinterpret_cast<uint4*>(lds + LdsLayout<R>::kSh)[tid] = make_uint4(gv, gv, gv, gv);
  if (walk_gap && tid < 128) reinterpret_cast<uint32_t*>(lds + walk_gap)[tid] = wv;
  __syncthreads();
}

template <int R>
struct Slice4T {
  const uint8_t* lds;
  uint32_t c3, c2, c1, c0;  // per lookup k = 0..3: its table's entry-0 offset + replica * 4 (bits 0-7 and 16-23)
  uint32_t g;               // shift tables + replica * 4
  // R = 16: lanes l and l + 16 share a replica, and a table's 16 replicas fill
  // 16 of the banks, so one lookup of every lane in one table is 2-way
  // conflicted. Instead each group of 16 lanes (q = (lane >> 4) & 3) does
  // lookup k on byte k ^ q: in every lookup instruction the four groups read
  // four different tables, which sit in different banks (entry(t, b) =
  // b * 256 + t * 64) - conflict-free. The byte position is then per lane, so
  // the v_perm selectors are registers (sel3..sel0) instead of immediates.
  uint32_t sel3 = 0, sel2 = 0, sel1 = 0, sel0 = 0;
  __device__ explicit Slice4T(const uint8_t* l) : lds(l) {
    const uint32_t r = (threadIdx.x & uint32_t(R - 1)) * 4u;
    const uint32_t q = R == 16 ? (threadIdx.x >> 4) & 3u : 0u;
    // lookup k reads byte k ^ q with table 3 - (k ^ q)
    c3 = LdsLayout<R>::entry(int(3 - (0 ^ q)), 0) + r;
    c2 = LdsLayout<R>::entry(int(3 - (1 ^ q)), 0) + r;
    c1 = LdsLayout<R>::entry(int(3 - (2 ^ q)), 0) + r;
    c0 = LdsLayout<R>::entry(int(3 - (3 ^ q)), 0) + r;
    if constexpr (R == 16) {
      sel3 = 0x0C020000u | ((4u + (0 ^ q)) << 8);
      sel2 = 0x0C020000u | ((4u + (1 ^ q)) << 8);
      sel1 = 0x0C020000u | ((4u + (2 ^ q)) << 8);
      sel0 = 0x0C020000u | ((4u + (3 ^ q)) << 8);
    }
    g = LdsLayout<R>::kSh + r;
  }
  // byte K of s at bits 8-15, the constant's bytes 0 and 2 around it (v_perm_b32:
  // selectors 0-3 pick bytes of the second operand, 4-7 of the first, 12 a zero)
  template <uint32_t K>
  __device__ __forceinline__ uint32_t lk(uint32_t s, uint32_t c, uint32_t sel) const {
    if constexpr (R == 16) return lds_word(lds, __builtin_amdgcn_perm(s, c, sel));
    else return lds_word(lds, __builtin_amdgcn_perm(s, c, 0x0C020000u | ((4u + K) << 8)));
  }
  // One slice-by-4 step on a register that already holds (crc ^ word), with the
  // NEXT word folded in: T3[b0] ^ T2[b1] ^ T1[b2] ^ T0[b3] ^ next (byte k of
  // the word is followed by 3 - k bytes: table 3 - k) - two 3-input XORs.
  __device__ __forceinline__ uint32_t mix(uint32_t s, uint32_t next) const {
    return x3(x3(lk<0>(s, c3, sel3), lk<1>(s, c2, sel2), lk<2>(s, c1, sel1)), lk<3>(s, c0, sel0), next);
  }
  __device__ __forceinline__ uint32_t word16(uint32_t s, u32x4_t w) const {
    return mix(mix(mix(mix(s ^ w[0], w[1]), w[2]), w[3]), 0u);
  }
  // shift over kGapBytes zeros, with `next` folded in
  __device__ __forceinline__ uint32_t gap(uint32_t s, uint32_t next) const {
    uint32_t r[8];
    if constexpr (R == 16) {
      // lanes 16-31 of each half-wave take table n ^ 1 where lanes 0-15 take
      // table n (the other bank half, LdsLayout<16>::gap_entry): on the
      // register with its nibbles swapped pairwise, nibble n is nibble n ^ 1
      const bool h = (threadIdx.x >> 4) & 1u;
      const uint32_t sw = ((s & 0x0F0F0F0Fu) << 4) | ((s >> 4) & 0x0F0F0F0Fu);
      const uint32_t t = h ? sw : s;
      const uint32_t ge = g + (h ? 64u : 0u), go = g + (h ? 0u : 64u);  // even / odd n
#pragma unroll
      for (int n = 0; n < 8; ++n)
        r[n] = lds_word(lds, (n & 1 ? go : ge) + uint32_t(n >> 1) * 2048u + ((t >> (4 * n)) & 15u) * 128u);
    } else {
#pragma unroll
      for (int n = 0; n < 8; ++n)
        r[n] = lds_word(lds, g + LdsLayout<R>::gap_entry(n, 0) + ((s >> (4 * n)) & 15u) * uint32_t(R * 4));
    }
    return x3(x3(x3(r[0], r[1], r[2]), r[3], r[4]), x3(r[5], r[6], r[7]), next);
  }
  // a ^ b ^ c in one v_bitop3_b32
  static __device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
};

// In-register 4x4 transpose across the 4 rows (16 lanes each) of a wave and 4
// registers: afterwards register q of lane m + 16 r holds what register r of
// lane m + 16 q held. permlane16_swap exchanges the odd rows of its first
// operand with the even rows of its second (swaps row bit 0 with register bit
// 0), permlane32_swap the upper half of the first with the lower half of the
// second (row bit 1 with register bit 1).
__device__ __forceinline__ void row_transpose(u32x4_t& r0, u32x4_t& r1, u32x4_t& r2, u32x4_t& r3) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const auto a = __builtin_amdgcn_permlane16_swap(r0[d], r1[d], false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(r2[d], r3[d], false, false);
    const auto c = __builtin_amdgcn_permlane32_swap(a[0], b[0], false, false);
    const auto e = __builtin_amdgcn_permlane32_swap(a[1], b[1], false, false);
    r0[d] = c[0];
    r2[d] = c[1];
    r1[d] = e[0];
    r3[d] = e[1];
  }
}

// One segment as the walker sees it (all fields wave-uniform).
struct Seg {
  const uint8_t* p;     // first byte
  int64_t len;          // bytes (16 KiB except a chunk's last)
  int64_t chunk, chunk_start, chunk_len, seg_start;
  uint32_t xrem;        // x^(8 * (chunk_len mod 16 KiB))
  uint16_t* out;        // the chunk's bf16 output (fused unpack), else nullptr
};

// A segment's raw CRC (at its own end) shifted to its chunk's end: what the
// segment adds to the chunk's raw CRC, so the fold is a plain XOR over the
// chunk's segments. Full segment k of a chunk with nfull full ones and a short
// tail of rem bytes moves over j = nfull - 1 - k segments (segpow, one entry
// per 10 bits of j) and rem bytes (xrem, skipped when rem = 0); the short tail
// segment already ends there. Every operand is wave-uniform (scalar ALU work,
// off the loads' critical path).
__device__ __forceinline__ uint32_t to_chunk_end(const Seg& sg, uint32_t s, const uint32_t* __restrict__ sc) {
  if (sg.len != kSegBytes) return s;
  const int64_t nfull = sg.chunk_len / kSegBytes, k = sg.seg_start / kSegBytes, j = nfull - 1 - k;
  uint32_t m = sc[kSegPow + (j & (kSegLevel - 1))];
  if (j >> 10) m = multmodp_unrolled(m, sc[kSegPow + kSegLevel + ((j >> 10) & (kSegLevel - 1))]);
  if (j >> 20) m = multmodp_unrolled(m, sc[kSegPow + 2 * kSegLevel + (j >> 20)]);
  if (sg.chunk_len % kSegBytes) m = multmodp_unrolled(m, sg.xrem);
  return multmodp_unrolled(m, s);
}

// Visit hooks: begin(seg) at a segment's start; operator()(w, e) per word of a
// partial segment; word(w, e, i) per word i (0-15, load order) of a full one;
// prefetch(seg, full) issues the loads a later segment's words need (called
// before its data loads, so waiting for them never waits for younger data
// loads) and advance() makes the prefetched values current.
struct NoVisit {
  __device__ void begin(const Seg&) {}
  __device__ void operator()(const u32x4_t&, int64_t) {}
  __device__ void word(const u32x4_t&, int64_t, int) {}
  __device__ void prefetch(const Seg&, bool) {}
  __device__ void advance() {}
};

// A segment shorter than 16 KiB (only ever its chunk's last): each lane takes
// the strided 16-B words j = lane (mod 64), CRCs each from a zero register and
// shifts it to the segment end with a pow16 constant; lane 0 adds the byte tail.
template <class Visit, class ST>
__device__ uint32_t slice_partial(const Seg& sg, const uint32_t* __restrict__ sc, const ST& st, int lane,
                                  Visit& visit) {
  const int64_t nw = sg.len >> 4;
  const u32x4_t* words = reinterpret_cast<const u32x4_t*>(sg.p);
  uint32_t acc = 0;
  for (int64_t j = lane; j < nw; j += 64) {
    const u32x4_t w = words[j];
    visit(w, sg.seg_start + 16 * j);
    acc ^= multmodp(sc[kPow + (nw - 1 - j)], st.word16(0, w));
  }
  acc = wave_xor(acc);
  if (lane == 0) {
    const uint8_t* tail = sg.p + (nw << 4);
    for (int64_t b = 0; b < (sg.len & 15); ++b) acc = sc[kT + ((acc ^ tail[b]) & 255)] ^ (acc >> 8);
  }
  return acc;
}

// The 16 loads of a segment's words go through a buffer resource whose size is
// 16 KiB for a full segment and 0 otherwise: an out-of-range buffer load
// returns zeros without touching memory, so every path issues the same loads
// and the compiler's vmcnt waits stay exact (with the prefetch under an `if`,
// it had to wait for ALL outstanding loads, the next segment's included).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seg_rsrc(const uint8_t* p, bool full) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0, full ? kSegBytes : 0, 0x00020000);
}
// load i = 4 * block + j: KiB j of the block, lane m + 16 r reads word r of piece 16 j + m (nt)
__device__ __forceinline__ u32x4_t seg_load(__amdgpu_buffer_rsrc_t r, int lo, int i) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (i >> 2) * kBlockBytes + (i & 3) * 1024 + lo, 0, 2);
}

// The CRC of one full segment whose 16 words w[] (as loaded) are in
// registers: per block, the visit sees the block's 4 words (as loaded, with
// their byte offsets in the chunk), then the transpose hands lane l its piece
// and the slice-by-4 chain runs; the lanes' registers are shifted to the
// segment end (lanec = x^(8*64*(63-lane))) and XOR-reduced.
template <class Visit, class ST>
__device__ __forceinline__ uint32_t seg_full(u32x4_t (&w)[4 * kBlocksPerSeg], const Seg& cur, const ST& st,
                                             Visit& visit, const uint32_t* __restrict__ lanec, int lo) {
  // s holds (register ^ next word) between steps: 16 mix steps per block,
  // the block's first word folded into the gap shift before it
  uint32_t s = 0;
#pragma unroll
  for (int b = 0; b < kBlocksPerSeg; ++b) {
#pragma unroll
    for (int j = 0; j < 4; ++j) visit.word(w[4 * b + j], cur.seg_start + b * kBlockBytes + j * 1024 + lo, 4 * b + j);
    row_transpose(w[4 * b], w[4 * b + 1], w[4 * b + 2], w[4 * b + 3]);
    s = b ? st.gap(s, w[4 * b][0]) : w[0][0];
#pragma unroll
    for (int x = 0; x < 16; ++x) s = st.mix(s, x < 15 ? w[4 * b + ((x + 1) >> 2)][(x + 1) & 3] : 0u);
    __builtin_amdgcn_sched_barrier(0);
  }
  return wave_xor_dpp(multmodp_unrolled(lanec[threadIdx.x & 63], s));
}


// Workgroup barrier for LDS hand-offs only: it waits for this wave's LDS
// operations, not for its global stores. __syncthreads() also drains vmcnt,
// which would hold every wave at the barrier until its bf16 stores are
// acknowledged (the workgroup's 80 KiB of LDS stay allocated meanwhile).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One segment per wave: the wave issues its segment's loads (and the scales)
// BEFORE the workgroup fills the LDS tables, then runs the segment and exits.
// On gfx9 one in-order counter (vmcnt) covers loads and stores, so a walking
// wave's next loads, issued behind its stores, cannot be waited for without
// those stores completing: a persistent read->write walk moved 512 MiB of bf16
// in 160 us where one-segment waves took 139 and a plain one-shot grid 131
// (bin/walkprobe, profiles/r4_walk*/). A CU streams many short-lived waves
// instead, and the table fill is paid per workgroup of WAVES segments.
// (The fill's own table reads, issued after the data loads, can only be
// waited for together with them; reading the tables into registers first and
// storing them after the data loads measured the same - 17.9 vs 18.0 us per
// 64 MiB chunk batched, profiles/r5_fill_order/: the CU's other workgroup
// already covers the fill.)
// Returns the segment's value at its chunk's end (to_chunk_end).
template <class Geo, class Visit, int R, int WAVES>
__device__ __forceinline__ uint32_t slice_once(const Geo& geo, int64_t g, bool have, const uint32_t* __restrict__ sc,
                                               uint8_t* lds, Visit& visit) {
  const int lane = threadIdx.x & 63;
  const int lo = kPieceBytes * (lane & 15) + 16 * (lane >> 4);
  Seg cur = have ? geo(g) : geo(0);
  const bool full = have && cur.len == kSegBytes;
  u32x4_t w[4 * kBlocksPerSeg];
  {
    const auto r = seg_rsrc(cur.p, full);
    visit.prefetch(cur, full);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4 * kBlocksPerSeg; ++i) {
      w[i] = seg_load(r, lo, i);
      __builtin_amdgcn_sched_barrier(0);
    }
    visit.advance();
  }
  load_lds_strided<R>(lds, sc);  // every wave joins the fill and its barrier
  if (!have) return 0;
  const Slice4T<R> st(lds);
  visit.begin(cur);
  uint32_t s;
  if (full) s = seg_full(w, cur, st, visit, sc + kLanePow, lo);
  else s = slice_partial(cur, sc, st, lane, visit);
  return to_chunk_end(cur, s, sc);
}

// Half a segment per wave, for the grid's last, partial round (see
// once_split): waves 2 m and 2 m + 1 of the workgroup take blocks 0-1 and 2-3
// of its segment m. Each half is a chain over its lanes' two pieces, shifted to
// the half's end like a segment (the per-lane constants are the same: a
// lane's last piece sits 64 * (63 - lane) bytes before its block's end); the
// first half moves over the second (x^(8 * 8 KiB) = pow16[512]) and the second
// hands its value over through LDS. A short segment is done whole by the
// first wave of the pair.
// (H is a template parameter so that every word index, and with it the scale
// register a word reads, is a compile-time constant: with a run-time half the
// scale array was indexed dynamically and moved to LDS, 36 KiB per workgroup.)
template <int H, class Visit>
__device__ __forceinline__ void half_load(const Seg& cur, bool full, Visit& visit, u32x4_t (&w)[8]) {
  const int lane = threadIdx.x & 63;
  const int lo = kPieceBytes * (lane & 15) + 16 * (lane >> 4);
  const auto r = seg_rsrc(cur.p, full);
  visit.prefetch(cur, full);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w[i] = seg_load(r, lo, 8 * H + i);
    __builtin_amdgcn_sched_barrier(0);
  }
  visit.advance();
}

template <int H, class Visit, int R>
__device__ __forceinline__ uint32_t half_seg(const Seg& cur, bool have, bool full, const uint32_t* __restrict__ sc,
                                             const uint8_t* lds, Visit& visit, u32x4_t (&w)[8]) {
  const int lane = threadIdx.x & 63;
  const int lo = kPieceBytes * (lane & 15) + 16 * (lane >> 4);
  const Slice4T<R> st(lds);
  uint32_t v = 0;
  if (have) {
    visit.begin(cur);
    if (full) {
      uint32_t s = 0;
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) {
        const int b = 2 * H + bb;
#pragma unroll
        for (int j = 0; j < 4; ++j) visit.word(w[4 * bb + j], cur.seg_start + b * kBlockBytes + j * 1024 + lo, 4 * b + j);
        row_transpose(w[4 * bb], w[4 * bb + 1], w[4 * bb + 2], w[4 * bb + 3]);
        s = bb ? st.gap(s, w[4 * bb][0]) : w[4 * bb][0];
#pragma unroll
        for (int x = 0; x < 16; ++x) s = st.mix(s, x < 15 ? w[4 * bb + ((x + 1) >> 2)][(x + 1) & 3] : 0u);
      }
      s = wave_xor_dpp(multmodp_unrolled(sc[kLanePow + lane], s));
      if constexpr (H == 0) s = multmodp_unrolled(sc[kPow + (kSegBytes / 2) / 16], s);
      v = s;
    } else if constexpr (H == 0) {
      v = slice_partial(cur, sc, st, lane, visit);
    }
  }
  return v;
}

// The second half's value goes through LDS word xch[stride * pair]: the
// second wave's own staging slot when there is one (two 80 KiB workgroups
// fill the CU's 160 KiB: not one more word to spare). Returns the pair's
// segment value (at its chunk's end) on the first wave, 0 on the second.
template <class Geo, class Visit, int R>
__device__ __forceinline__ uint32_t slice_half(const Geo& geo, int64_t g, bool have, const uint32_t* __restrict__ sc,
                                               uint8_t* lds, Visit& visit, uint32_t* xch, int stride) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = wave & 1;
  const Seg cur = have ? geo(g) : geo(0);
  const bool full = have && cur.len == kSegBytes;
  u32x4_t w[8];
  if (h) half_load<1>(cur, full, visit, w);
  else half_load<0>(cur, full, visit, w);
  load_lds_strided<R>(lds, sc);  // every wave joins the fill and its barrier
  const uint32_t v = h ? half_seg<1, Visit, R>(cur, have, full, sc, lds, visit, w)
                       : half_seg<0, Visit, R>(cur, have, full, sc, lds, visit, w);
  if (h == 1 && lane == 0) xch[stride * (wave >> 1)] = v;
  lds_barrier();
  return h == 0 && have ? to_chunk_end(cur, v ^ xch[stride * (wave >> 1)], sc) : 0;
}

// 16 e4m3fn values (one 16-B word) times their power-of-two block scale -> 16 bf16 (32 B in o).
__device__ inline void unpack16_regs(const u32x4_t& w, float s, uint32_t (&o)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = fp8x2_to_bf16x2<false>(w[i], s);
    o[2 * i + 1] = fp8x2_to_bf16x2<true>(w[i], s);
  }
}
__device__ inline void unpack16_nt(const u32x4_t& w, float s, uint4* __restrict__ dst) {
  uint32_t o[8];
  unpack16_regs(w, s, o);
  __builtin_nontemporal_store(u32x4_t{o[0], o[1], o[2], o[3]}, reinterpret_cast<u32x4_t*>(dst));
  __builtin_nontemporal_store(u32x4_t{o[4], o[5], o[6], o[7]}, reinterpret_cast<u32x4_t*>(dst) + 1);
}

// A wave's 2 KiB of bf16 from one loaded word (lane m + 16 r holds output bytes
// [128 m + 32 r, +32)) written as two fully coalesced 1 KiB stores (lane i:
// bytes 16 i of each half) through a 1 KiB LDS slot of the wave: the lanes of
// half h (m in 8h..8h+7) write their 32 B, every lane reads back 16 B and
// stores. Stored directly, each of the two store instructions covers the 2 KiB
// at half density (16 B in every 32). One wave's LDS operations run in issue
// order, so no barrier is needed between its writes and reads.
// The slot's 64 16-B granules are swizzled (g -> g ^ ((g >> 3) & 7)): the
// writers of one 16-lane group (granules 8 m + 2 r, m = 0..7) then hit 8
// distinct bank quads instead of 2 (4-way conflicts: 29 M conflict cycles per
// 512 MiB, profiles/r3_kernels; the & 6 of rounds 3-5 left pairs of them in
// one quad of the 32-lane half), and the readers (granule = lane) stay distinct.
// The stores are nontemporal: the output is written once and never read back,
// so it has no business in L2 or the Infinity Cache (5.04 -> 5.39-5.43 TB/s at
// 512 MiB, profiles/r4_nt).
__device__ __forceinline__ uint32_t swz(uint32_t g) { return g ^ ((g >> 3) & 7u); }
__device__ __forceinline__ void store_staged(const uint32_t (&o)[8], uint8_t* slot, uint4* __restrict__ region) {
  const int lane = threadIdx.x & 63, m = lane & 15, r = lane >> 4;
  uint4* g = reinterpret_cast<uint4*>(slot);  // granules
  const uint32_t w0 = swz(uint32_t(8 * (m & 7) + 2 * r)), w1 = swz(uint32_t(8 * (m & 7) + 2 * r + 1));
  const uint4* rd = g + swz(uint32_t(lane));
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if ((m >> 3) == h) {
      g[w0] = make_uint4(o[0], o[1], o[2], o[3]);
      g[w1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_nontemporal_store(*reinterpret_cast<const u32x4_t*>(rd), reinterpret_cast<u32x4_t*>(region) + 64 * h + lane);
    __builtin_amdgcn_wave_barrier();
  }
}

// Fused verify + unpack of fp8-packed chunks (core/fp8.h layout
// [q: n bytes][scales: n/BLOCK f32] per chunk): while computing each segment's
// CRC, words in the q region are dequantized and written as bf16 (on the
// words as loaded: each wave store instruction writes 2 whole KiB). Every
// packed byte is read once from HBM.
//
// Scales: a full segment's 16 KiB / BLOCK scales are loaded with the
// segment's data, issued before it (lane l, register r: scale l + 64 r of the
// segment), and each word takes its scale from the owning lane with
// ds_bpermute (the register index is uniform per word: a word's scales never
// straddle 64). Loading each word's scale where it is used made every use wait
// for all older loads (vmcnt counts in order): 3.93 -> 4.12 TB/s in the round-2
// walk (profiles/r2_fused_ahead).
template <int BLOCK>
struct UnpackVisit {
  static constexpr int kR = kSegBytes / BLOCK >= 64 ? kSegBytes / BLOCK / 64 : 1;  // scale registers
  // BLOCK 32 would hold 16 scale registers and spill: it keeps the per-word load
  static constexpr bool kAhead = kR <= 4;
  int64_t n_q = 0;
  const float* scales = nullptr;
  uint16_t* obase = nullptr;
  uint8_t* slot = nullptr;  // this wave's 1 KiB of LDS
  float cs[kAhead ? kR : 1] = {}, ns[kAhead ? kR : 1] = {};  // scales of the current / next full segment
  __device__ void begin(const Seg& sg) {
    n_q = sg.chunk_len / (BLOCK + 4) * BLOCK;  // q bytes (= elements) of this chunk
    scales = reinterpret_cast<const float*>(sg.p - sg.seg_start + n_q);
    obase = sg.out;
  }
  __device__ void operator()(const u32x4_t& w, int64_t e) {  // e: byte offset in chunk = element index in q
    if (e < n_q) unpack16_nt(w, scales[e / BLOCK], reinterpret_cast<uint4*>(obase + e));
  }
  __device__ void prefetch(const Seg& sg, bool full) {
    if constexpr (!kAhead) return;
    const int64_t nq = sg.chunk_len / (BLOCK + 4) * BLOCK;
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(sg.p - sg.seg_start + nq), 0,
                                                     full ? int(nq / BLOCK * 4) : 0, 0x00020000);
    const int first = int(sg.seg_start / BLOCK) + int(threadIdx.x & 63);
#pragma unroll
    for (int k = 0; k < (kAhead ? kR : 1); ++k)  // past the chunk's scales (the q/scale boundary): zeros
      ns[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (first + 64 * k) * 4, 0, 0));
  }
  __device__ void advance() {
#pragma unroll
    for (int k = 0; k < (kAhead ? kR : 1); ++k) cs[k] = ns[k];
  }
  // word i of a full segment (all lanes active): lane m + 16 r covers bytes
  // lo = 64 m + 16 r of each KiB, scale (KiB offset + lo) / BLOCK
  __device__ void word(const u32x4_t& w, int64_t e, int i) {
    if constexpr (!kAhead) {
      (*this)(w, e);
      return;
    }
    const int lane = threadIdx.x & 63;
    const int base = ((i >> 2) * kBlockBytes + (i & 3) * 1024) / BLOCK;
    const int from = (base & 63) + (64 * (lane & 15) + 16 * (lane >> 4)) / BLOCK;
    const float s = __builtin_bit_cast(
        float, __builtin_amdgcn_ds_bpermute(from * 4, __builtin_bit_cast(int, cs[kAhead ? (base >> 6) : 0])));
    // the KiB this word covers: wave-uniform (lane offsets 0..1008 inside it)
    const int64_t kib = e - (64 * (lane & 15) + 16 * (lane >> 4));
    if (kib + 1024 <= n_q) {
      uint32_t o[8];
      unpack16_regs(w, s, o);
      store_staged(o, slot, reinterpret_cast<uint4*>(obase + kib));
      return;
    }
    if (e < n_q) unpack16_nt(w, s, reinterpret_cast<uint4*>(obase + e));
  }
};

// ---- geometry of a launch: which bytes each segment covers, and per item
// (a chunk whose CRC32C is one result) its segment count, init/xorout term and
// result word.

// `bytes` cut into chunks of `chunk_bytes` (one item per chunk); with an
// unpack, chunk c's bf16 goes to out + c * out_chunk_elems.
struct ChunkGeo {
  const uint8_t* src;
  int64_t bytes, chunk_bytes, spc;
  uint32_t xrem_full, xrem_last;  // x^(8 * (len mod 16 KiB)) of a full chunk / the last chunk
  uint32_t init_full, init_last;  // init/xorout terms of a full chunk / the last chunk
  uint32_t* crc_out;              // crc_out[c]: chunk c's CRC32C
  uint16_t* out;                  // bf16 output (fused), else nullptr
  int64_t out_chunk_elems;
  __device__ Seg operator()(int64_t g) const {
    const int64_t c = g / spc, k = g - c * spc;
    Seg s;
    s.chunk = c;
    s.chunk_start = c * chunk_bytes;
    s.chunk_len = min(chunk_bytes, bytes - s.chunk_start);
    s.seg_start = k * kSegBytes;
    s.p = src + s.chunk_start + s.seg_start;
    s.len = min(int64_t(kSegBytes), s.chunk_len - s.seg_start);
    s.xrem = s.chunk_len == chunk_bytes ? xrem_full : xrem_last;
    s.out = out ? out + c * out_chunk_elems : nullptr;
    return s;
  }
  __device__ int64_t item_segs(int64_t c) const {
    return (min(chunk_bytes, bytes - c * chunk_bytes) + kSegBytes - 1) / kSegBytes;
  }
  __device__ uint32_t item_init(int64_t c) const { return (c + 1) * chunk_bytes <= bytes ? init_full : init_last; }
  __device__ uint32_t* item_out(int64_t c) const { return crc_out + c; }
};

// Up to kCrcBatchMax independent items (the chunks one P2P group or one
// staging batch landed), each 16-B aligned, any length.
struct BatchGeo {
  int n;
  int64_t seg_base[kCrcBatchMax + 1];  // prefix sums of the items' segment counts
  const uint8_t* src[kCrcBatchMax];
  int64_t bytes[kCrcBatchMax];
  uint32_t xrem[kCrcBatchMax];  // x^(8 * (bytes mod 16 KiB))
  uint32_t init[kCrcBatchMax];
  uint32_t* crc_out[kCrcBatchMax];
  uint16_t* out[kCrcBatchMax];  // bf16 output of each item (fused)
  __device__ Seg operator()(int64_t g) const {
    int j = 0;
    while (g >= seg_base[j + 1]) ++j;  // wave-uniform, at most kCrcBatchMax steps
    const int64_t k = g - seg_base[j];
    Seg s;
    s.chunk = j;
    s.chunk_start = 0;
    s.chunk_len = bytes[j];
    s.seg_start = k * kSegBytes;
    s.p = src[j] + s.seg_start;
    s.len = min(int64_t(kSegBytes), bytes[j] - s.seg_start);
    s.xrem = xrem[j];
    s.out = out[j];
    return s;
  }
  __device__ int64_t item_segs(int64_t j) const { return seg_base[j + 1] - seg_base[j]; }
  __device__ uint32_t item_init(int64_t j) const { return init[j]; }
  __device__ uint32_t* item_out(int64_t j) const { return crc_out[j]; }
};

// ---- the fold, inside the kernel (no second launch). A chunk's raw CRC is
// the XOR of its segments' values (each already shifted to the chunk end).
// Per item the workspace holds one 64-bit word {acc (low half), count (high
// half)}: every workgroup XORs the value of its segments of the item into acc
// (one device-scope atomic per run of its waves that share an item), then
// adds its segment count to count, both on that same word; the workgroup
// whose add completes the item's count has the complete acc in the add's
// returned value, zeroes the word and writes raw ^ init. Words are back at 0
// when the launch ends, so a workspace zeroed once serves every later launch
// on its stream.
// Ordering by the memory model with relaxed atomics only: a workgroup's XOR
// and add are RMWs of one location in program order, so the XOR precedes the
// add in that location's modification order (write-write coherence); the
// completing add comes after every other add, so after every XOR, and an RMW
// reads the value just before it - acc complete. (Round 5 put acc and count in
// two words with an asm dependency between the atomics; release on the count
// add / acquire in the completer made that formal but the release's L2
// write-back of the fused kernel's bf16 stores took it from 18.0 to 32.5 us per
// chunk batched, profiles/r6_verify.) The separate fold launch this replaces
// cost 8.4-9.6 us per 64 MiB chunk in the round-4 engine traces
// (profiles/r4_profile), a quarter of the verify.
template <class Geo>
__device__ __forceinline__ void fold_add(const Geo& geo, int64_t item, uint32_t x, uint32_t n, uint32_t* acc) {
  auto* a = reinterpret_cast<unsigned long long*>(acc) + item;
  __hip_atomic_fetch_xor(a, static_cast<unsigned long long>(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long old =
      __hip_atomic_fetch_add(a, static_cast<unsigned long long>(n) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (int64_t((old >> 32) + n) == geo.item_segs(item)) {
    __hip_atomic_store(a, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *geo.item_out(item) = uint32_t(old) ^ geo.item_init(item);
  }
}

// Thread 0 of a workgroup: its waves' values (item < 0: none) in runs of equal item.
template <class Geo, int WAVES>
__device__ __forceinline__ void fold_workgroup(const Geo& geo, const uint32_t* v, const int64_t* item, uint32_t* acc) {
  int64_t cur = -1;
  uint32_t x = 0, n = 0;
  for (int w = 0; w < WAVES; ++w) {
    if (item[w] < 0) continue;
    if (item[w] != cur) {
      if (cur >= 0) fold_add(geo, cur, x, n, acc);
      cur = item[w];
      x = 0;
      n = 0;
    }
    x ^= v[w];
    ++n;
  }
  if (cur >= 0) fold_add(geo, cur, x, n, acc);
}

// The verify kernel: one 16 KiB segment per wave (slice_once), 512-thread
// workgroups with 16 table replicas (72 KiB of LDS, + 8 KiB of bf16 staging
// with an unpack): two workgroups per CU, so one fills its tables and waits
// for its first loads while the other computes. Workgroups [split_block, ..)
// take half segments (once_split). BLOCK: the fp8 scale block of the fused
// unpack (the CRC-only check is crc_walk_kernel below).
// Round 4 measured this shape against the alternatives for the fused path
// (profiles/r4_nt, r4_kernels_final: 5.3-5.5 TB/s at 512 MiB vs 4.66 for the
// persistent walk with staged stores, 3.6-4.1 for the walk's other store
// forms, 4.3 for split CRC/unpack waves); those variants were removed from
// the library. Batching several landed chunks into one launch is what makes
// it fast at the engine's chunk size: one 64 MiB chunk alone is 264
// workgroups, less than one per CU slot, and ran at 3.0 TB/s (profiles/r4_sizes).
template <class Geo, int BLOCK>
__global__ void __launch_bounds__(kWaves16 * 64) __attribute__((amdgpu_waves_per_eu(4)))
verify_once16_kernel(const Geo geo, int64_t total_segs, int64_t split_block, const uint32_t* __restrict__ sc,
                     uint32_t* __restrict__ acc) {
  static_assert(BLOCK > 0, "fused only");
  using Visit = UnpackVisit<BLOCK>;
  // Per wave after the tables: its 1 KiB bf16 staging slot. Bytes 16-31 of a
  // wave's slot carry its fold value and item to thread 0 (its staging is done
  // by then; word 0 may hold a half-pair hand-over). Two 80 KiB workgroups
  // fill the CU's 160 KiB: not one more byte to spare.
  constexpr uint32_t kSlot = 1024;
  __shared__ uint4 lds_raw[(LdsLayout<16>::kBytes + kWaves16 * kSlot) / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  uint8_t* slots = lds + LdsLayout<16>::kBytes;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Visit v{};
  v.slot = slots + wave * kSlot;
  uint32_t val;
  int64_t item = -1;
  if (int64_t(blockIdx.x) < split_block) {
    const int64_t g = int64_t(blockIdx.x) * kWaves16 + wave;
    const bool have = g < total_segs;
    val = slice_once<Geo, Visit, 16, kWaves16>(geo, g, have, sc, lds, v);
    if (have) item = geo(g).chunk;
  } else {
    const int64_t g = split_block * kWaves16 + (int64_t(blockIdx.x) - split_block) * (kWaves16 / 2) + (wave >> 1);
    const bool have = g < total_segs;
    // pair m hands over in word 0 of wave 2 m + 1's slot
    val = slice_half<Geo, Visit, 16>(geo, g, have, sc, lds, v, reinterpret_cast<uint32_t*>(slots + kSlot),
                                     int(2 * kSlot / 4));
    if (have && (wave & 1) == 0) item = geo(g).chunk;
  }
  if (lane == 0) {
    *reinterpret_cast<uint32_t*>(slots + wave * kSlot + 16) = val;
    *reinterpret_cast<int64_t*>(slots + wave * kSlot + 24) = item;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    uint32_t vs[kWaves16];
    int64_t its[kWaves16];
#pragma unroll
    for (int w = 0; w < kWaves16; ++w) {
      vs[w] = *reinterpret_cast<const uint32_t*>(slots + w * kSlot + 16);
      its[w] = *reinterpret_cast<const int64_t*>(slots + w * kSlot + 24);
    }
    fold_workgroup<Geo, kWaves16>(geo, vs, its, acc);
  }
}

// The CRC-only check: a walk. With no stores there is no in-order vmcnt to
// fear (the reason the fused kernel runs one segment per wave), so one
// 1024-thread workgroup per CU fills its 32-replica (conflict-free) tables
// ONCE and its 16 waves walk the workgroup's contiguous range of segments:
// wave w takes g0 + w, g0 + w + 16, ..., and loads block b of its next
// segment as soon as block b of the current one is consumed (pinned with
// sched_barrier: left alone, the compiler sinks those loads behind the math),
// so 16 KiB stay in flight per wave. One segment per wave with the tables
// filled per 8 segments measured 3.8 TB/s for CRC alone (profiles/r5_verify/);
// this walk 5.67 TB/s on 1 GiB and 12.6 us per 64 MiB chunk in 16-chunk
// launches, 0.94-1.0 TB/s on the 32 CUs of the verify stream with peers
// (profiles/r5_walk/). Issuing the first segment's loads before the table
// fill (slice_once's order) measured slower here - 28 vs 24 us for a lone
// chunk, 13.3 vs 12.6 per chunk in a batch (verify_bench_*loads_before_fill):
// the fill's own table loads then wait behind them in the in-order vmcnt.
// Reading the tables into registers first, then the segment, then storing
// the tables, measured neutral: 25.9 us lone, 12.6 batched, 5.78 TB/s on
// 1 GiB (profiles/r5_fill_order/).
// The fold: a wave accumulates its values while its item does not change and
// hands each run to the workgroup's LDS slot of that item (ds atomics); at
// the end the workgroup adds one value per item to the global {acc, count}
// (fold_add) - one pair of device-scope atomics per (workgroup, item), 16
// per 64 MiB item in a 16-chunk batch, instead of one per 8 segments.
constexpr int kWalkSlots = 256;
// Bytes between the end of a lane's piece in block 3 of segment g and the
// start of its piece in block 0 of segment g + kWalkWaves (the walk's stride).
constexpr int64_t kWalkGapBytes = int64_t(kWalkWaves) * kSegBytes - (kBlocksPerSeg - 1) * kBlockBytes - kPieceBytes;

// s shifted over kWalkGapBytes zeros with `next` folded in (the 16-entry
// nibble tables at LDS byte `base`: every lane reads one of 16 consecutive
// words per table, so at most one address per bank - no replicas needed).
// s = 0 gives next: a run's first segment takes the same path.
__device__ __forceinline__ uint32_t walk_gap(const uint8_t* lds, uint32_t base, uint32_t s, uint32_t next) {
  uint32_t r[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) r[n] = lds_word(lds, base + uint32_t(n) * 64u + ((s >> (4 * n)) & 15u) * 4u);
  using S = Slice4T<32>;
  return S::x3(S::x3(S::x3(r[0], r[1], r[2]), r[3], r[4]), S::x3(r[5], r[6], r[7]), next);
}

// One wave's walk over segments g = first, first + kWalkWaves, ... < end.
// While its next segment is a full one of the same item, a lane carries its
// CRC state on over the zeros to its piece there (walk_gap: 8 lookups)
// instead of shifting it to the segment end and reducing the wave (a 32-step
// GF(2) multiply and a DPP reduction, ~30 % of a segment's VALU work). At a
// run's end (item change, partial segment or end of range) the state is
// shifted and reduced once, and sink(seg, value, segments) on lane 0 gets the
// run's value at the item's end: CRC is linear, so the other waves' segments
// between (zeros here) add their own values. `gap`: walk_gap's LDS tables.
template <class Geo, class Sink>
__device__ __forceinline__ void crc_walk(const Geo& geo, int64_t first, int64_t end, const uint32_t* __restrict__ sc,
                                         const Slice4T<32>& st, uint32_t gap, uint32_t* prog, Sink sink) {
  const int lane = threadIdx.x & 63;
  const int lo = kPieceBytes * (lane & 15) + 16 * (lane >> 4);
  int64_t g = first;
  if (g >= end) return;
  NoVisit visit;
  Seg cur = geo(g);
  // invariant at the loop top: w holds cur's words if cur is a full segment
  u32x4_t w[4 * kBlocksPerSeg];
  {
    const auto r = seg_rsrc(cur.p, cur.len == kSegBytes);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4 * kBlocksPerSeg; ++i) {  // in order: every path issues w[0..15] oldest first
      w[i] = seg_load(r, lo, i);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  uint32_t run = 0;  // the lane's state carried from the run's previous segment (0: none)
  uint32_t nrun = 0;  // segments in the run so far (wave-uniform)
  uint32_t mine = 0;  // segments this wave has done
  for (; g < end; g += kWalkWaves) {
    const int64_t gn = g + kWalkWaves;
    Seg nxt = cur;  // no next segment: loads against an empty resource
    bool nfull = false;
    if (gn < end) {
      nxt = geo(gn);
      nfull = nxt.len == kSegBytes;
    }
    const auto rn = seg_rsrc(nxt.p, nfull);
    uint32_t s;
    bool more;  // the run goes on into nxt
    if (cur.len == kSegBytes) {
      const uint32_t rowc = sc[kLanePow + lane];
      s = 0;
#pragma unroll
      for (int b = 0; b < kBlocksPerSeg; ++b) {
        row_transpose(w[4 * b], w[4 * b + 1], w[4 * b + 2], w[4 * b + 3]);
        s = b ? st.gap(s, w[4 * b][0]) : walk_gap(st.lds, gap, run, w[0][0]);
#pragma unroll
        for (int x = 0; x < 16; ++x) s = st.mix(s, x < 15 ? w[4 * b + ((x + 1) >> 2)][(x + 1) & 3] : 0u);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) w[4 * b + j] = seg_load(rn, lo, 4 * b + j);
        __builtin_amdgcn_sched_barrier(0);
      }
      ++nrun;
      more = nfull && nxt.chunk == cur.chunk;
      if (more) {
        run = s;
      } else {
        run = 0;
        s = wave_xor_dpp(multmodp_unrolled(rowc, s));
      }
    } else {  // a partial segment: a run of its own (the one before it ended at the item's full segments)
      s = slice_partial(cur, sc, st, lane, visit);
      nrun = 1;
      more = false;
    }
    if (!more) {
      if (lane == 0) sink(cur, to_chunk_end(cur, s, sc), nrun);
      nrun = 0;
    }
    // Progress-balanced issue: a wave behind its workgroup's average raises its
    // priority. Left to the arbiter, which favors older waves, the last wave of
    // a workgroup finished 7-20 us after the first (profiles/r6_walk_anatomy).
    ++mine;
    uint32_t tot = 0;
    if (lane == 0) tot = atomicAdd(prog, 1u) + 1u;
    tot = __builtin_amdgcn_readfirstlane(tot);
    if (mine * kWalkWaves < tot) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(0);
    if (cur.len != kSegBytes) {  // (rare) w did not take the next segment's words yet
#pragma unroll
      for (int i = 0; i < 4 * kBlocksPerSeg; ++i) {
        w[i] = seg_load(rn, lo, i);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    cur = nxt;
  }
}

template <class Geo>
__global__ void __launch_bounds__(kWalkWaves * 64) __attribute__((amdgpu_waves_per_eu(4)))
crc_walk_kernel(const Geo geo, int64_t total_segs, int64_t per_wg, const uint32_t* __restrict__ sc,
                uint32_t* __restrict__ acc) {
  constexpr uint32_t kFold = LdsLayout<32>::kBytes, kGapT = kFold + kWalkSlots * 8, kProg = kGapT + 8 * 16 * 4;
  __shared__ uint4 lds_raw[(kProg + 16) / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  uint32_t* fx = reinterpret_cast<uint32_t*>(lds + kFold);  // per item slot: XOR
  uint32_t* fn = fx + kWalkSlots;                           // ... and segment count
  const int64_t g0 = int64_t(blockIdx.x) * per_wg, g1 = min(g0 + per_wg, total_segs);
  if (g0 >= g1) return;  // whole workgroup
  constexpr int NT = kWalkWaves * 64;
  static_assert(2 * kWalkSlots <= NT, "one slot word per thread");
  const int tid = threadIdx.x;
  if (tid < 2 * kWalkSlots) fx[tid] = 0;
  uint32_t* prog = reinterpret_cast<uint32_t*>(lds + kProg);  // segments the workgroup's waves have done
  if (tid == 0) *prog = 0;
  const int64_t first_item = geo(g0).chunk;
  load_lds<32, NT>(lds, sc, kGapT);  // once per workgroup; its barrier also publishes the slots
  const Slice4T<32> st(lds);
  // two LDS atomics per run of a wave's segments in one item (the host keeps a range within kWalkSlots items)
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));  // uniform: g and its Seg in SGPRs
  crc_walk(geo, g0 + wave, g1, sc, st, kGapT, prog, [=](const Seg& sg, uint32_t v, uint32_t n) {
    const int slot = int(sg.chunk - first_item);
    atomicXor(&fx[slot], v);
    atomicAdd(&fn[slot], n);
  });
  lds_barrier();
  const int64_t nslots = geo(g1 - 1).chunk - first_item + 1;
  for (int64_t t = tid; t < nslots; t += NT)
    if (fn[t]) fold_add(geo, first_item + t, fx[t], fn[t], acc);
}

// Per-device constant tables (one upload per device, before any RCCL traffic:
// crc32c_warm at engine set-up).
//
// Uploaded WITHOUT a host-synchronous copy: a hipMemcpy here ran on the null
// stream in the middle of a session (the first CRC of a rank that starts by
// receiving), waited for the comm lanes' RCCL kernels, and hung a rank whose
// peers waited for it (profiles/r3_multihost/). The tables go to pinned host
// memory and are copied with hipMemcpyAsync on the caller's stream; an event
// recorded behind the copy orders any later user on another stream.
struct ConstEntry {
  uint32_t* d = nullptr;
  hipEvent_t ready = nullptr;
};
struct DeviceConsts {
  std::mutex mu;
  std::map<int, ConstEntry> by_device;
};
DeviceConsts g_consts;

ConstEntry upload_consts(const std::vector<uint32_t>& h, hipStream_t s) {
  void *d = nullptr, *hp = nullptr;
  const size_t n = h.size() * 4;
  if (hipMalloc(&d, n) != hipSuccess) return {};
  if (hipHostMalloc(&hp, n, hipHostMallocDefault) != hipSuccess) return {};  // kept: the copy may still read it
  memcpy(hp, h.data(), n);
  ConstEntry e;
  e.d = static_cast<uint32_t*>(d);
  if (hipMemcpyAsync(d, hp, n, hipMemcpyHostToDevice, s) != hipSuccess) return {};
  if (hipEventCreateWithFlags(&e.ready, hipEventDisableTiming) != hipSuccess) return {};
  if (hipEventRecord(e.ready, s) != hipSuccess) return {};
  return e;
}

// Tables for use on stream s (a no-op wait once their upload has run).
uint32_t* use_on(const ConstEntry& e, hipStream_t s) {
  if (!e.d) return nullptr;
  if (hipStreamWaitEvent(s, e.ready, 0) != hipSuccess) return nullptr;
  return e.d;
}

uint32_t* device_consts(hipStream_t s) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_consts.mu);
  auto it = g_consts.by_device.find(dev);
  if (it != g_consts.by_device.end()) return use_on(it->second, s);
  std::vector<uint32_t> T(16 * 256), h(kConstWords);
  crc32c_slice16_tables(T.data());
  for (int i = 0; i < 4 * 256; ++i) h[size_t(kT + i)] = T[size_t(i)];
  const uint32_t xg = crc32c_xpow8n(kGapBytes);
  for (int n = 0; n < 8; ++n)
    for (uint32_t v = 0; v < 16; ++v) h[size_t(kGap + n * 16 + int(v))] = crc32c_multmodp(xg, v << (4 * n));
  const uint32_t xw = crc32c_xpow8n(uint64_t(kWalkGapBytes));
  for (int n = 0; n < 8; ++n)
    for (uint32_t v = 0; v < 16; ++v) h[size_t(kWalkGap + n * 16 + int(v))] = crc32c_multmodp(xw, v << (4 * n));
  for (int m = 0; m < 1024; ++m) h[size_t(kPow + m)] = crc32c_xpow8n(uint64_t(16) * uint64_t(m));
  for (int l = 0; l < 64; ++l) h[size_t(kLanePow + l)] = crc32c_xpow8n(uint64_t(kPieceBytes) * uint64_t(63 - l));
  // segpow level L, entry i: x^(8 * 16 KiB * i * 1024^L)
  for (int L = 0; L < kSegLevels; ++L) {
    const uint64_t step = uint64_t(kSegBytes) << (10 * L);
    const uint32_t xs = crc32c_xpow8n(step);
    h[size_t(kSegPow + L * kSegLevel)] = 0x80000000u;  // x^0
    for (int i = 1; i < kSegLevel; ++i)
      h[size_t(kSegPow + L * kSegLevel + i)] = crc32c_multmodp(xs, h[size_t(kSegPow + L * kSegLevel + i - 1)]);
  }
  const ConstEntry e = upload_consts(h, s);
  if (!e.d) return nullptr;
  g_consts.by_device[dev] = e;
  return e.d;
}

// Resident verify workgroups per CU, cached per device.
int once16_per_cu() {
  static std::mutex mu;
  static std::map<int, int> by_device;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  if (auto it = by_device.find(dev); it != by_device.end()) return it->second;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, verify_once16_kernel<ChunkGeo, 128>, kWaves16 * 64, 0) !=
      hipSuccess)
    per_cu = 2;
  return by_device[dev] = std::max(1, per_cu);
}

int device_cus() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  return cus;
}

// Grid with its last, partial round of workgroups done in half segments
// (slice_half). Every workgroup lasts about as long, so with W workgroups on
// S slots the kernel takes ceil(W / S) rounds even when the last holds only a
// few: 16896 segments (512 MiB of bf16 packed) are 2112 workgroups on 512
// slots, 4.125 rounds. Cutting the last round's segments in halves gives
// twice the workgroups at half the length, so a last round up to half full
// ends in half the time. W <= S / 2: every segment in halves (twice the
// parallelism); otherwise no split. S counts the slots of the CUs the stream
// may use (`cus`: a CU-masked verify stream passes its CU count; 0 = all).
struct OnceGrid {
  int64_t split_block;  // workgroups [0, split_block) take whole segments
  unsigned blocks;
};
OnceGrid once_split(int64_t total_segs, int cus) {
  const int dc = device_cus();
  const int64_t W = (total_segs + kWaves16 - 1) / kWaves16;
  const int64_t S = int64_t(once16_per_cu()) * (cus > 0 ? std::min(cus, dc) : dc);
  int64_t full = W;
  if (W <= S) full = 2 * W <= S ? 0 : W;
  else if (const int64_t tail = W % S; tail && 2 * tail <= S) full = W - tail;
  const int64_t half_segs = std::max<int64_t>(0, total_segs - full * kWaves16);
  return OnceGrid{full, unsigned(full + (half_segs + kWaves16 / 2 - 1) / (kWaves16 / 2))};
}

int64_t segs_of(int64_t n) { return (n + kSegBytes - 1) / kSegBytes; }

// Fewest segments of any item but the last (bounds the items one walk range spans).
int64_t min_item_segs(const ChunkGeo& g) { return g.spc; }
int64_t min_item_segs(const BatchGeo&) { return 1 << 20; }  // at most kCrcBatchMax items in all

template <class Geo>
hipError_t launch(const Geo& geo, int64_t total_segs, int block, const uint32_t* consts, void* ws, hipStream_t s,
                  int cus) {
  if (total_segs <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(ws) & 7) return hipErrorInvalidValue;  // 64-bit fold words
  auto* acc = static_cast<uint32_t*>(ws);
  if (block == 0) {
    // CRC only: one walking workgroup per CU the stream may use, each a
    // contiguous range of segments (at least one per wave)
    const int dc = device_cus();
    const int64_t wgs = std::max<int64_t>(
        1, std::min<int64_t>(cus > 0 ? std::min(cus, dc) : dc, (total_segs + kWalkWaves - 1) / kWalkWaves));
    // a range spans at most kWalkSlots items: one LDS slot each (items of
    // at least min_item_segs segments; a batch holds at most kCrcBatchMax)
    const int64_t per_wg = std::min((total_segs + wgs - 1) / wgs, (kWalkSlots - 2) * min_item_segs(geo));
    crc_walk_kernel<Geo><<<dim3(unsigned((total_segs + per_wg - 1) / per_wg)), dim3(kWalkWaves * 64), 0, s>>>(
        geo, total_segs, per_wg, consts, acc);
    return hipGetLastError();
  }
  const OnceGrid og = once_split(total_segs, cus);
  const dim3 grid(og.blocks), tpb(kWaves16 * 64);
  switch (block) {
    case 32: verify_once16_kernel<Geo, 32><<<grid, tpb, 0, s>>>(geo, total_segs, og.split_block, consts, acc); break;
    case 64: verify_once16_kernel<Geo, 64><<<grid, tpb, 0, s>>>(geo, total_segs, og.split_block, consts, acc); break;
    case 128: verify_once16_kernel<Geo, 128><<<grid, tpb, 0, s>>>(geo, total_segs, og.split_block, consts, acc); break;
    case 256: verify_once16_kernel<Geo, 256><<<grid, tpb, 0, s>>>(geo, total_segs, og.split_block, consts, acc); break;
    case 512: verify_once16_kernel<Geo, 512><<<grid, tpb, 0, s>>>(geo, total_segs, og.split_block, consts, acc); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}


// A ChunkGeo over `bytes` in `chunk_bytes` chunks (the caller checked alignment).
hipError_t chunk_geo(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* crc_out, ChunkGeo* g,
                     int64_t* total_segs) {
  const int64_t spc = segs_of(chunk_bytes);
  if (spc > kMaxSegs) return hipErrorInvalidValue;
  const int64_t nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  const int64_t last_len = bytes - (nchunks - 1) * chunk_bytes;
  auto xrem = [](int64_t len) { return crc32c_xpow8n(uint64_t(len % kSegBytes)); };
  *g = ChunkGeo{static_cast<const uint8_t*>(src), bytes, chunk_bytes, spc, xrem(chunk_bytes), xrem(last_len),
                crc32c_init_term(uint64_t(chunk_bytes)), crc32c_init_term(uint64_t(last_len)), crc_out, nullptr, 0};
  *total_segs = (nchunks - 1) * spc + segs_of(last_len);
  return hipSuccess;
}

// Appends item (src, bytes) to a BatchGeo.
hipError_t batch_add(BatchGeo& a, const void* src, int64_t bytes, uint32_t* crc_out, uint16_t* out) {
  if (reinterpret_cast<uintptr_t>(src) & 15) return hipErrorInvalidValue;
  const int64_t spc = segs_of(bytes);
  if (spc > kMaxSegs || a.n >= kCrcBatchMax) return hipErrorInvalidValue;
  const int j = a.n++;
  a.src[j] = static_cast<const uint8_t*>(src);
  a.bytes[j] = bytes;
  a.xrem[j] = crc32c_xpow8n(uint64_t(bytes % kSegBytes));
  a.init[j] = crc32c_init_term(uint64_t(bytes));
  a.crc_out[j] = crc_out;
  a.out[j] = out;
  a.seg_base[j + 1] = a.seg_base[j] + spc;
  return hipSuccess;
}

// Packed bytes of `src_len` bf16 source bytes (one chunk's worth) with `block` scales.
int64_t packed_of(int64_t src_len, int block) { return src_len / 2 + src_len / 2 / block * 4; }

bool valid_block(int block) { return block == 32 || block == 64 || block == 128 || block == 256 || block == 512; }

}  // namespace

hipError_t crc32c_warm(hipStream_t s) { return device_consts(s) ? hipSuccess : hipErrorOutOfMemory; }

size_t crc32c_workspace_bytes(int64_t bytes, int64_t chunk_bytes) {
  if (bytes <= 0 || chunk_bytes <= 0) return 16;
  const int64_t nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  return size_t((nchunks * 8 + 15) / 16 * 16);
}

size_t crc32c_batch_workspace_bytes() { return size_t(kCrcBatchMax) * 8; }

hipError_t crc32c_chunks(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                         hipStream_t s, int cus) {
  if (bytes <= 0) return hipSuccess;
  if (chunk_bytes <= 0 || (reinterpret_cast<uintptr_t>(src) & 15)) return hipErrorInvalidValue;
  // One chunk may have any length: only a chunk's last segment is partial, and
  // it takes a byte tail. Several chunks need a 16-B multiple so that every
  // chunk starts 16-B aligned.
  if (bytes <= chunk_bytes) chunk_bytes = bytes;
  else if (chunk_bytes % 16) return hipErrorInvalidValue;
  const uint32_t* consts = device_consts(s);
  if (!consts) return hipErrorOutOfMemory;
  ChunkGeo geo;
  int64_t total = 0;
  if (hipError_t e = chunk_geo(src, bytes, chunk_bytes, out, &geo, &total); e != hipSuccess) return e;
  return launch(geo, total, 0, consts, workspace, s, cus);
}

hipError_t crc32c_batch(const CrcItem* items, int n, void* workspace, hipStream_t s, int cus) {
  if (n <= 0) return hipSuccess;
  if (n > kCrcBatchMax) return hipErrorInvalidValue;
  const uint32_t* consts = device_consts(s);
  if (!consts) return hipErrorOutOfMemory;
  BatchGeo a{};
  for (int i = 0; i < n; ++i)
    if (items[i].bytes > 0)
      if (hipError_t e = batch_add(a, items[i].src, items[i].bytes, items[i].out, nullptr); e != hipSuccess) return e;
  if (a.n == 0) return hipSuccess;
  for (int j = a.n; j < kCrcBatchMax; ++j) a.seg_base[j + 1] = a.seg_base[a.n];
  return launch(a, a.seg_base[a.n], 0, consts, workspace, s, cus);
}

hipError_t fp8_verify_unpack(const void* packed, int64_t src_bytes, int64_t src_chunk, int block, uint16_t* out,
                             uint32_t* crc_out, void* workspace, hipStream_t s, int cus) {
  if (src_bytes <= 0) return hipSuccess;
  if (src_chunk <= 0 || src_chunk % 4096 || !valid_block(block) || src_bytes % (2 * block) ||
      (reinterpret_cast<uintptr_t>(packed) & 15) || (reinterpret_cast<uintptr_t>(out) & 15))
    return hipErrorInvalidValue;
  const int64_t pchunk = packed_of(src_chunk, block);
  const int64_t full = src_bytes / src_chunk, tail = src_bytes % src_chunk;
  const int64_t bytes = full * pchunk + (tail ? packed_of(tail, block) : 0);
  const uint32_t* consts = device_consts(s);
  if (!consts) return hipErrorOutOfMemory;
  ChunkGeo geo;
  int64_t total = 0;
  if (hipError_t e = chunk_geo(packed, bytes, pchunk, crc_out, &geo, &total); e != hipSuccess) return e;
  geo.out = out;
  geo.out_chunk_elems = src_chunk / 2;
  return launch(geo, total, block, consts, workspace, s, cus);
}

hipError_t fp8_verify_unpack_batch(const FusedItem* items, int n, int block, void* workspace, hipStream_t s, int cus) {
  if (n <= 0) return hipSuccess;
  if (n > kCrcBatchMax || !valid_block(block)) return hipErrorInvalidValue;
  const uint32_t* consts = device_consts(s);
  if (!consts) return hipErrorOutOfMemory;
  BatchGeo a{};
  for (int i = 0; i < n; ++i) {
    const FusedItem& it = items[i];
    if (it.src_len <= 0) continue;
    if (it.src_len % (2 * block) || (reinterpret_cast<uintptr_t>(it.out) & 15)) return hipErrorInvalidValue;
    if (hipError_t e = batch_add(a, it.packed, packed_of(it.src_len, block), it.crc_out, it.out); e != hipSuccess)
      return e;
  }
  if (a.n == 0) return hipSuccess;
  for (int j = a.n; j < kCrcBatchMax; ++j) a.seg_base[j + 1] = a.seg_base[a.n];
  return launch(a, a.seg_base[a.n], block, consts, workspace, s, cus);
}

}  // namespace kern
}  // namespace dissem
