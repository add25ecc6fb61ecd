// Per-chunk CRC32C on gfx950 (receiver-side verification of every landed chunk).
//
// CRC is a serial recurrence, so the kernel works with raw (un-inverted) CRC
// registers, which are linear over GF(2):
//   raw(A || B) = shift(raw(A), |B|) xor raw(B),  shift(r, L) = r * x^(8L) mod P.
// Decomposition:
//  * a chunk is cut into 16 KiB segments; one wave owns a segment;
//  * a segment is 4 blocks of 4 KiB, and lane l owns the contiguous 64-B piece
//    l of every block. Within a piece the classic slice-by-4 recurrence runs
//    (s ^= word; s = T3[b0] ^ T2[b1] ^ T1[b2] ^ T0[b3]): one table lookup per
//    byte. Between its pieces a lane's register crosses the 4032 bytes of the
//    other lanes as zeros: a fixed GF(2)-linear map, 8 nibble lookups;
//  * each lane's CRC is shifted to the END OF ITS SEGMENT with one GF(2)
//    multiply by a per-lane constant (x^(8*64*(63-lane))), then the lanes are
//    XOR-reduced with cross-lane shuffles: a segment's value is its raw CRC;
//  * the wave then shifts that value to the END OF ITS CHUNK - x^(8*16 KiB*j)
//    from one table indexed by the segments that follow it, then x^(8*rem)
//    for a chunk whose last segment is short (wave-uniform products);
//  * a second, small kernel (one workgroup per chunk) XORs a chunk's segment
//    values and adds the init/xorout term, writing the standard CRC32C.
// The constants depend on nothing but the segment geometry (chunks up to
// 1 GiB): one upload per device, never a per-length table (a length-keyed
// table grew with every new piece size and re-allocated mid-session).
// The result is the exact CRC32C of each chunk for any chunk length that is a
// multiple of 16 (the buffer's final chunk may have any length).
//
// Loads stay coalesced: each 16-B load instruction of a wave reads one whole
// KiB (lane m + 16 r: word r of piece 16 j + m of KiB j), and a 4x4 register
// transpose across the wave's 4 rows (v_permlane16_swap / v_permlane32_swap,
// 16 VALU per 64 B of lane data) hands lane l its piece l. Loading the pieces
// directly (every lane 16 B of its own piece per instruction: 64 separate
// 64-B spans) reads at 3.5-4.0 TB/s against 6.8 for whole KiBs in the same
// 16-KiB-per-wave shape (kern::read_seg probe, profiles/r2_crc_ab).
//
// LDS layout (MI355X_MICROARCH.md, LDS): a ds_read_b32 is served in two groups
// of 32 lanes over 32 banks, and data-dependent indices into a plain table
// conflict (2x the useful LDS cycles in round 1, profiles/r1_counters). Every
// table entry is stored 32 times, replica r in bank r, and lane l reads replica
// l & 31: conflict-free by construction. The 4 byte tables take 128 KiB (two
// per 64 KiB: entry b at row b * 256 B, odd table at +128 B), so the address
// of byte k of s is (b << 8) | (half * 128 + replica * 4) | (pair << 16): ONE
// v_perm_b32 of s with a per-lane constant, then the ds_read_b32. With the
// 16 KiB of shift tables that is 144 KiB: one 1024-thread workgroup per CU.
//
// History (profiles/r2_crc_ab): nibble tables on strided 16-B words (40
// lookups per 16 B; 2.7 TB/s on 1 GiB, 31 us per 64 MiB chunk), the same on
// byte-addressed nibble tables with a rolling prefetch (3.3 TB/s), an MFMA
// GF(2) product (2.3 TB/s), slice-by-4 on directly loaded pieces (3.1 TB/s)
// and with 4 independent recurrences per lane (2.3-2.5 TB/s) all lost to this
// kernel: 5.76 TB/s on 1 GiB (186.5 us, kernel trace; the same load shape with
// no math reads at 6.8 TB/s), 16.6 us + 4.5 us fold per single 64 MiB chunk.
// Per 16 KiB segment a wave issues ~256 v_perm + ~130 v_bitop3 (3-input XORs)
// for the lookups, 64 permlane swaps and ~160 VALU for the branch-free shift to
// the chunk end (the divergent multiply loop cost 212 us per GiB).
// Two recurrences per lane (blocks 0-1 and 2-3, joined by an 8 KiB shift
// table in the last 16 KiB of LDS) measured 229 us: the chain latency is not
// what bounds it. Round 4 (fused kernel, profiles/r4_chains): four chains per
// lane, one per block, joined by 4096-byte shifts, measured the same as one
// chain (160.4 vs 157.9 us main kernel at 512 MiB, 29.6 vs 30.3 at 64 MiB):
// the ~9 us a launch pays over the same kernel without CRC math is the first
// and last waves' ~600 VALU + 256 LDS lookups per lane per segment with
// nothing to hide behind, not the length of the dependency chain.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <cstring>
#include <mutex>
#include <tuple>
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
constexpr uint32_t kShLds = 131072;                     // shift tables after the byte tables
constexpr uint32_t kLdsBytes = kShLds + 8 * 16 * 128;   // 144 KiB
constexpr uint32_t kStageBytes = 16 * 1024;              // fused unpack: 1 KiB output staging per wave
constexpr int kThreads = 1024;                          // one workgroup per CU, 4 waves per SIMD
constexpr int kWaves = kThreads / 64;
// Global constants: [T: 4 x 256 (T[k][v]: byte v then k zero bytes)]
// [gap: 8 x 16 nibble tables of the kGapBytes shift][pow16: 1024 (x^(8*16 m))]
// [lanepow: 64 (x^(8*64*(63-l)): lane l's last piece to its segment end)]
// [segpow: kMaxSegs (x^(8*16 KiB*j))].
constexpr int kMaxSegs = 65536;  // segments per chunk: chunks up to 1 GiB
constexpr int kT = 0, kGap = 1024, kPow = kGap + 128, kLanePow = kPow + 1024, kSegPow = kLanePow + 64,
              kConstWords = kSegPow + kMaxSegs;

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
  // byte table t, entry b, replica r
  static __device__ __forceinline__ uint32_t entry(int t, int b) {
    return R == 32 ? uint32_t(t >> 1) * 65536u + uint32_t(b) * 256u + uint32_t(t & 1) * 128u
                   : uint32_t(b) * 256u + uint32_t(t) * 64u;
  }
};
static_assert(LdsLayout<32>::kBytes == kLdsBytes, "144 KiB layout");

template <int R = 32>
__device__ inline void load_lds(uint8_t* lds, const uint32_t* __restrict__ sc) {
  constexpr int Q = R / 4;  // 16-B stores per entry
  for (int i = threadIdx.x; i < 4 * 256 * Q; i += blockDim.x) {
    const int e = i / Q, q = i % Q, t = e >> 8, b = e & 255;
    const uint32_t v = sc[kT + e];
    reinterpret_cast<uint4*>(lds + LdsLayout<R>::entry(t, b))[q] = make_uint4(v, v, v, v);
  }
  for (int i = threadIdx.x; i < 8 * 16 * Q; i += blockDim.x) {
    const int e = i / Q, q = i % Q;
    const uint32_t v = sc[kGap + e];
    reinterpret_cast<uint4*>(lds + LdsLayout<R>::kSh + uint32_t(e) * uint32_t(R * 4))[q] = make_uint4(v, v, v, v);
  }
  __syncthreads();
}

template <int R>
struct Slice4T {
  const uint8_t* lds;
  uint32_t c3, c2, c1, c0;  // per table t: its entry-0 offset + replica * 4 (bits 0-7 and 16-23)
  uint32_t g;               // shift tables + replica * 4
  __device__ explicit Slice4T(const uint8_t* l) : lds(l) {
    const uint32_t r = (threadIdx.x & uint32_t(R - 1)) * 4u;
    c0 = LdsLayout<R>::entry(0, 0) + r;
    c1 = LdsLayout<R>::entry(1, 0) + r;
    c2 = LdsLayout<R>::entry(2, 0) + r;
    c3 = LdsLayout<R>::entry(3, 0) + r;
    g = LdsLayout<R>::kSh + r;
  }
  // byte k of s at bits 8-15, the constant's bytes 0 and 2 around it (v_perm_b32:
  // selectors 0-3 pick bytes of the second operand, 4-7 of the first, 12 a zero)
  template <uint32_t K>
  __device__ __forceinline__ uint32_t lk(uint32_t s, uint32_t c) const {
    return lds_word(lds, __builtin_amdgcn_perm(s, c, 0x0C020000u | ((4u + K) << 8)));
  }
  // One slice-by-4 step on a register that already holds (crc ^ word), with the
  // NEXT word folded in: T3[b0] ^ T2[b1] ^ T1[b2] ^ T0[b3] ^ next (byte k of
  // the word is followed by 3 - k bytes: table 3 - k) - two 3-input XORs.
  __device__ __forceinline__ uint32_t mix(uint32_t s, uint32_t next) const {
    return x3(x3(lk<0>(s, c3), lk<1>(s, c2), lk<2>(s, c1)), lk<3>(s, c0), next);
  }
  __device__ __forceinline__ uint32_t word16(uint32_t s, u32x4_t w) const {
    return mix(mix(mix(mix(s ^ w[0], w[1]), w[2]), w[3]), 0u);
  }
  // shift over kGapBytes zeros, with `next` folded in
  __device__ __forceinline__ uint32_t gap(uint32_t s, uint32_t next) const {
    uint32_t r[8];
#pragma unroll
    for (int n = 0; n < 8; ++n)
      r[n] = lds_word(lds, g + uint32_t(n) * uint32_t(16 * R * 4) + ((s >> (4 * n)) & 15u) * uint32_t(R * 4));
    return x3(x3(x3(r[0], r[1], r[2]), r[3], r[4]), x3(r[5], r[6], r[7]), next);
  }
  // a ^ b ^ c in one v_bitop3_b32
  static __device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
};
using Slice4 = Slice4T<32>;

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
};

// A segment's raw CRC (at its own end) shifted to its chunk's end: what the
// segment adds to the chunk's raw CRC, so the fold is a plain XOR over the
// chunk's segments. Full segment k of a chunk with nfull full ones and a short
// tail of rem bytes moves over (nfull - 1 - k) segments (segpow) and rem bytes
// (xrem, skipped when rem = 0); the short tail segment already ends there.
// Every operand is wave-uniform: one or two 32-step products per segment, off
// the loads' critical path (the separate shift-and-fold launch took 7.4 us
// per 512 MiB, profiles/r4_kernels).
__device__ __forceinline__ uint32_t to_chunk_end(const Seg& sg, uint32_t s, const uint32_t* __restrict__ sc) {
  if (sg.len != kSegBytes) return s;
  const int64_t nfull = sg.chunk_len / kSegBytes, k = sg.seg_start / kSegBytes;
  uint32_t m = sc[kSegPow + (nfull - 1 - k)];
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
// segment end (lanec = x^(8*64*(63-lane))) and XOR-reduced. `between(b)` runs
// after block b (the persistent walk issues the next segment's block-b loads
// there). CRC = false (diagnostic only) keeps the visits and drops the math.
template <class Visit, bool CRC, class ST, class Between>
__device__ __forceinline__ uint32_t seg_full(u32x4_t (&w)[4 * kBlocksPerSeg], const Seg& cur, const ST& st,
                                             Visit& visit, const uint32_t* __restrict__ lanec, int lo,
                                             Between between) {
  // s holds (register ^ next word) between steps: 16 mix steps per block,
  // the block's first word folded into the gap shift before it
  uint32_t s = 0;
#pragma unroll
  for (int b = 0; b < kBlocksPerSeg; ++b) {
#pragma unroll
    for (int j = 0; j < 4; ++j) visit.word(w[4 * b + j], cur.seg_start + b * kBlockBytes + j * 1024 + lo, 4 * b + j);
    if constexpr (CRC) {
      row_transpose(w[4 * b], w[4 * b + 1], w[4 * b + 2], w[4 * b + 3]);
      s = b ? st.gap(s, w[4 * b][0]) : w[0][0];
#pragma unroll
      for (int x = 0; x < 16; ++x) s = st.mix(s, x < 15 ? w[4 * b + ((x + 1) >> 2)][(x + 1) & 3] : 0u);
    }
    __builtin_amdgcn_sched_barrier(0);
    between(b);
  }
  if constexpr (CRC) s = wave_xor_dpp(multmodp_unrolled(lanec[threadIdx.x & 63], s));
  return s;
}

// Every wave walks segments g = wave, wave + nwaves, ... (geo(g) -> Seg) and
// writes seg_out[g]: the segment's raw CRC shifted to its chunk's end. A wave
// that owns several segments loads block b of the next one as soon as block b
// of the current one is consumed (pinned with sched_barrier: left alone, the
// compiler sinks those loads behind the math), so 16 KiB stay in flight per
// wave. Visit sees every 16-B word (as loaded, before the transpose) with its
// byte offset in the chunk.
// CRC = false (diagnostic A/B only: its segment values are garbage) keeps the
// walk, the loads and the visits and drops the CRC math.
template <class Geo, class Visit, bool CRC = true>
__device__ __forceinline__ void slice_walk(const Geo& geo, int64_t total_segs, const uint32_t* __restrict__ sc,
                                           const Slice4& st, Visit& visit, uint32_t* __restrict__ seg_out,
                                           int waves_per_wg = kWaves) {
  const int lane = threadIdx.x & 63;
  const int64_t wave =
      __builtin_amdgcn_readfirstlane(int(blockIdx.x * waves_per_wg + ((threadIdx.x >> 6) % waves_per_wg)));
  const int64_t nwaves = int64_t(gridDim.x) * waves_per_wg;
  const int lo = kPieceBytes * (lane & 15) + 16 * (lane >> 4);
  int64_t g = wave;
  if (g >= total_segs) return;
  Seg cur = geo(g);
  // invariant at the loop top: w holds cur's words if cur is a full segment
  u32x4_t w[4 * kBlocksPerSeg];
  {
    const auto r = seg_rsrc(cur.p, cur.len == kSegBytes);
    visit.prefetch(cur, cur.len == kSegBytes);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4 * kBlocksPerSeg; ++i) {  // in order: every path issues w[0..15] oldest first
      w[i] = seg_load(r, lo, i);
      __builtin_amdgcn_sched_barrier(0);
    }
    visit.advance();
  }
  for (; g < total_segs; g += nwaves) {
    const int64_t gn = g + nwaves;
    Seg nxt = cur;  // no next segment: loads against an empty resource
    bool nfull = false;
    if (gn < total_segs) {
      nxt = geo(gn);
      nfull = nxt.len == kSegBytes;
    }
    const auto rn = seg_rsrc(nxt.p, nfull);
    visit.begin(cur);
    uint32_t s;
    if (cur.len == kSegBytes) {
      // (written out rather than through seg_full: the fused kernel sits at the
      // 128-VGPR cap here, and the helper's form spilled 8 bytes per lane)
      const uint32_t rowc = sc[kLanePow + lane];
      s = 0;
#pragma unroll
      for (int b = 0; b < kBlocksPerSeg; ++b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) visit.word(w[4 * b + j], cur.seg_start + b * kBlockBytes + j * 1024 + lo, 4 * b + j);
        if constexpr (CRC) {
          row_transpose(w[4 * b], w[4 * b + 1], w[4 * b + 2], w[4 * b + 3]);
          s = b ? st.gap(s, w[4 * b][0]) : w[0][0];
#pragma unroll
          for (int x = 0; x < 16; ++x) s = st.mix(s, x < 15 ? w[4 * b + ((x + 1) >> 2)][(x + 1) & 3] : 0u);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (b == 0) {  // the next segment's scales go out ahead of its data
          visit.prefetch(nxt, nfull);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) w[4 * b + j] = seg_load(rn, lo, 4 * b + j);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (CRC) s = wave_xor_dpp(multmodp_unrolled(rowc, s));
    } else {
      s = slice_partial(cur, sc, st, lane, visit);
    }
    if (lane == 0) seg_out[g] = to_chunk_end(cur, s, sc);
    if (cur.len != kSegBytes) {  // (rare) w did not take the next segment's words yet
      visit.prefetch(nxt, nfull);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4 * kBlocksPerSeg; ++i) {
        w[i] = seg_load(rn, lo, i);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    visit.advance();
    cur = nxt;
  }
}

// One segment per wave (no walk): the wave issues its segment's loads (and
// the scales) BEFORE the workgroup fills the LDS tables, then runs the
// segment and exits. On gfx9 one in-order counter (vmcnt) covers loads and
// stores, so a walking wave's next loads, issued behind its stores, cannot be
// waited for without those stores completing: a persistent read->write walk
// moved 512 MiB of bf16 in 160 us where one-segment waves took 139 and a
// plain one-shot grid 131 (bin/walkprobe, profiles/r4_walk*/). Here a CU
// streams many short-lived waves instead, and the table fill is paid per
// workgroup of kWaves segments.
template <class Geo, class Visit, bool CRC = true, int R = 32, int WAVES = kWaves>
__device__ __forceinline__ void slice_once(const Geo& geo, int64_t total_segs, const uint32_t* __restrict__ sc,
                                           uint8_t* lds, Visit& visit, uint32_t* __restrict__ seg_out) {
  const int lane = threadIdx.x & 63;
  const int64_t g = int64_t(blockIdx.x) * WAVES + (threadIdx.x >> 6);
  const bool have = g < total_segs;
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
  load_lds<R>(lds, sc);  // every wave joins the fill and its barrier
  if (!have) return;
  const Slice4T<R> st(lds);
  visit.begin(cur);
  uint32_t s;
  if (full) s = seg_full<Visit, CRC>(w, cur, st, visit, sc + kLanePow, lo, [](int) {});
  else s = slice_partial(cur, sc, st, lane, visit);
  if (lane == 0) seg_out[g] = to_chunk_end(cur, s, sc);
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

template <int H, class Visit, bool CRC, int R>
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
        if constexpr (CRC) {
          row_transpose(w[4 * bb], w[4 * bb + 1], w[4 * bb + 2], w[4 * bb + 3]);
          s = bb ? st.gap(s, w[4 * bb][0]) : w[4 * bb][0];
#pragma unroll
          for (int x = 0; x < 16; ++x) s = st.mix(s, x < 15 ? w[4 * bb + ((x + 1) >> 2)][(x + 1) & 3] : 0u);
        }
      }
      if constexpr (CRC) {
        s = wave_xor_dpp(multmodp_unrolled(sc[kLanePow + lane], s));
        if constexpr (H == 0) s = multmodp_unrolled(sc[kPow + (kSegBytes / 2) / 16], s);
      }
      v = s;
    } else if constexpr (H == 0) {
      v = slice_partial(cur, sc, st, lane, visit);
    }
  }
  return v;
}

// The second half's value goes through LDS word xch[stride * pair]: the
// second wave's own staging slot when there is one (two 80 KiB workgroups
// fill the CU's 160 KiB: not one more word to spare).
template <class Geo, class Visit, bool CRC = true, int R = 32, int WAVES = kWaves>
__device__ __forceinline__ void slice_half(const Geo& geo, int64_t total_segs, int64_t g0,
                                           const uint32_t* __restrict__ sc, uint8_t* lds, Visit& visit,
                                           uint32_t* __restrict__ seg_out, uint32_t* xch, int stride) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = wave & 1;
  const int64_t g = g0 + (wave >> 1);
  const bool have = g < total_segs;
  const Seg cur = have ? geo(g) : geo(0);
  const bool full = have && cur.len == kSegBytes;
  u32x4_t w[8];
  if (h) half_load<1>(cur, full, visit, w);
  else half_load<0>(cur, full, visit, w);
  load_lds<R>(lds, sc);  // every wave joins the fill and its barrier
  const uint32_t v = h ? half_seg<1, Visit, CRC, R>(cur, have, full, sc, lds, visit, w)
                       : half_seg<0, Visit, CRC, R>(cur, have, full, sc, lds, visit, w);
  if (h == 1 && lane == 0) xch[stride * (wave >> 1)] = v;
  __syncthreads();
  if (h == 0 && have && lane == 0) seg_out[g] = to_chunk_end(cur, v ^ xch[stride * (wave >> 1)], sc);
}

// `bytes` cut into chunks of `chunk_bytes`.
struct ChunkGeo {
  const uint8_t* src;
  int64_t bytes, chunk_bytes, spc;
  uint32_t xrem_full, xrem_last;  // x^(8 * (len mod 16 KiB)) of a full chunk / the last chunk
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
    return s;
  }
};

__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
crc32c_segments_kernel(const ChunkGeo geo, int64_t total_segs, const uint32_t* __restrict__ sc,
                       uint32_t* __restrict__ seg_out) {
  __shared__ uint4 lds_raw[kLdsBytes / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  load_lds(lds, sc);
  const Slice4 st(lds);
  NoVisit v;
  slice_walk(geo, total_segs, sc, st, v, seg_out);
}

// 16 e4m3fn values (one 16-B word) times their power-of-two block scale -> 16 bf16 (32 B in o).
__device__ inline void unpack16_regs(const u32x4_t& w, float s, uint32_t (&o)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = fp8x2_to_bf16x2<false>(w[i], s);
    o[2 * i + 1] = fp8x2_to_bf16x2<true>(w[i], s);
  }
}
template <bool NT = false>
__device__ inline void unpack16(const u32x4_t& w, float s, uint4* __restrict__ dst) {
  uint32_t o[8];
  unpack16_regs(w, s, o);
  if constexpr (NT) {
    __builtin_nontemporal_store(u32x4_t{o[0], o[1], o[2], o[3]}, reinterpret_cast<u32x4_t*>(dst));
    __builtin_nontemporal_store(u32x4_t{o[4], o[5], o[6], o[7]}, reinterpret_cast<u32x4_t*>(dst) + 1);
  } else {
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
  }
}

// A wave's 2 KiB of bf16 from one loaded word (lane m + 16 r holds output bytes
// [128 m + 32 r, +32)) written as two fully coalesced 1 KiB stores (lane i:
// bytes 16 i of each half) through a 1 KiB LDS slot of the wave: the lanes of
// half h (m in 8h..8h+7) write their 32 B, every lane reads back 16 B and
// stores. Stored directly, each of the two store instructions covers the 2 KiB
// at half density (16 B in every 32). One wave's LDS operations run in issue
// order, so no barrier is needed between its writes and reads.
// The slot's 64 16-B granules are swizzled (g -> g ^ ((g >> 3) & 6)): the
// writers of one 16-lane group (granules 8 m + 2 r, m = 0..7) then hit 8
// distinct bank quads instead of 2 (4-way conflicts: 29 M conflict cycles per
// 512 MiB, profiles/r3_kernels), and the readers (granule = lane) stay distinct.
__device__ __forceinline__ uint32_t swz(uint32_t g) { return g ^ ((g >> 3) & 6u); }
template <bool NT = false>
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
    if constexpr (NT)
      __builtin_nontemporal_store(*reinterpret_cast<const u32x4_t*>(rd), reinterpret_cast<u32x4_t*>(region) + 64 * h + lane);
    else
      region[64 * h + lane] = *rd;
    __builtin_amdgcn_wave_barrier();
  }
}

// Fused verify + unpack of fp8-packed chunks (core/fp8.h layout
// [q: n bytes][scales: n/BLOCK f32] per chunk): while computing each segment's
// CRC, words in the q region are dequantized and written as bf16 (on the
// words as loaded: each wave store instruction writes 2 whole KiB). Every
// packed byte is read once from HBM.
//
// Scales: a full segment's 16 KiB / BLOCK scales are loaded one segment ahead
// (lane l, register r: scale l + 64 r of the segment), issued before that
// segment's data loads, and each word takes its scale from the owning lane with
// ds_bpermute (the register index is uniform per word: a word's scales never
// straddle 64). Loading each word's scale where it is used made every use wait
// for all older loads - the next segment's prefetch included (vmcnt counts in
// order): 3.93 -> 4.12 TB/s (profiles/r2_fused_ahead). Nontemporal bf16 stores
// (NT) measured slower in the round-2 walk, whose lanes stored half-dense 16-B
// pieces (3.61 TB/s, profiles/r2_fused_nt), and still lose there (store 14:
// 3.6); the staged, whole-KiB stores of the one-segment-per-wave kernel gain
// from them: 5.04 -> 5.39-5.43 TB/s at 512 MiB, 5.37-5.67 -> 5.92-6.13 at
// 4 GiB (profiles/r4_nt): the output is written once and never read back, so
// it has no business in L2 or the Infinity Cache.
template <int BLOCK, bool STAGE = false, bool NT = false>
struct UnpackVisit {
  static constexpr int kR = kSegBytes / BLOCK >= 64 ? kSegBytes / BLOCK / 64 : 1;  // scale registers
  // BLOCK 32 would hold 16 scale registers and spill: it keeps the per-word load
  static constexpr bool kAhead = kR <= 4;
  int64_t out_chunk_elems;
  uint16_t* out;
  const uint8_t* src;
  int64_t n_q = 0;
  const float* scales = nullptr;
  uint16_t* obase = nullptr;
  uint8_t* slot = nullptr;  // STAGE: this wave's 1 KiB of LDS
  float cs[kAhead ? kR : 1] = {}, ns[kAhead ? kR : 1] = {};  // scales of the current / next full segment
  __device__ void begin(const Seg& sg) {
    n_q = sg.chunk_len / (BLOCK + 4) * BLOCK;  // q bytes (= elements) of this chunk
    scales = reinterpret_cast<const float*>(src + sg.chunk_start + n_q);
    obase = out + sg.chunk * out_chunk_elems;
  }
  __device__ void operator()(const u32x4_t& w, int64_t e) {  // e: byte offset in chunk = element index in q
    if (e < n_q) unpack16<NT>(w, scales[e / BLOCK], reinterpret_cast<uint4*>(obase + e));
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
    if constexpr (STAGE) {
      // the KiB this word covers: wave-uniform (lane offsets 0..1008 inside it)
      const int64_t kib = e - (64 * (lane & 15) + 16 * (lane >> 4));
      if (kib + 1024 <= n_q) {
        uint32_t o[8];
        unpack16_regs(w, s, o);
        store_staged<NT>(o, slot, reinterpret_cast<uint4*>(obase + kib));
        return;
      }
    }
    if (e < n_q) unpack16<NT>(w, s, reinterpret_cast<uint4*>(obase + e));
  }
};

template <int BLOCK, bool STAGE, bool CRC = true>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
verify_unpack_segments_kernel(const ChunkGeo geo, int64_t total_segs, int64_t out_chunk_elems,
                              const uint32_t* __restrict__ sc, uint32_t* __restrict__ seg_out,
                              uint16_t* __restrict__ out) {
  __shared__ uint4 lds_raw[(kLdsBytes + (STAGE ? kStageBytes : 0)) / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  load_lds(lds, sc);
  const Slice4 st(lds);
  UnpackVisit<BLOCK, STAGE> v{out_chunk_elems, out, geo.src};
  v.slot = lds + kLdsBytes + (threadIdx.x >> 6) * 1024;
  slice_walk<ChunkGeo, UnpackVisit<BLOCK, STAGE>, CRC>(geo, total_segs, sc, st, v, seg_out);
}

// store = 5: one segment per wave (slice_once), the grid as large as the work.
template <int BLOCK, bool CRC = true>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
verify_unpack_once_kernel(const ChunkGeo geo, int64_t total_segs, int64_t out_chunk_elems,
                          const uint32_t* __restrict__ sc, uint32_t* __restrict__ seg_out,
                          uint16_t* __restrict__ out) {
  __shared__ uint4 lds_raw[(kLdsBytes + kStageBytes) / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  UnpackVisit<BLOCK, true> v{out_chunk_elems, out, geo.src};
  v.slot = lds + kLdsBytes + (threadIdx.x >> 6) * 1024;
  slice_once<ChunkGeo, UnpackVisit<BLOCK, true>, CRC>(geo, total_segs, sc, lds, v, seg_out);
}

// store = 7: one segment per wave, 512-thread workgroups with 16 table
// replicas (72 KiB + 8 KiB of staging): two workgroups per CU, so one fills
// its tables and waits for its first loads while the other computes.
constexpr int kWaves16 = 8;
template <int BLOCK, bool CRC = true, bool STAGE = true, bool NT = false>
__global__ void __launch_bounds__(kWaves16 * 64) __attribute__((amdgpu_waves_per_eu(4)))
verify_unpack_once16_kernel(const ChunkGeo geo, int64_t total_segs, int64_t split_block, int64_t out_chunk_elems,
                            const uint32_t* __restrict__ sc, uint32_t* __restrict__ seg_out,
                            uint16_t* __restrict__ out) {
  __shared__ uint4 lds_raw[(LdsLayout<16>::kBytes + (STAGE ? kWaves16 * 1024 : 0)) / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  UnpackVisit<BLOCK, STAGE, NT> v{out_chunk_elems, out, geo.src};
  v.slot = lds + LdsLayout<16>::kBytes + (threadIdx.x >> 6) * 1024;
  if (int64_t(blockIdx.x) < split_block) {
    slice_once<ChunkGeo, UnpackVisit<BLOCK, STAGE, NT>, CRC, 16, kWaves16>(geo, total_segs, sc, lds, v, seg_out);
  } else {
    const int64_t g0 = split_block * kWaves16 + (int64_t(blockIdx.x) - split_block) * (kWaves16 / 2);
    if constexpr (STAGE) {  // pair m hands over in word 0 of wave 2 m + 1's slot
      slice_half<ChunkGeo, UnpackVisit<BLOCK, STAGE, NT>, CRC, 16, kWaves16>(
          geo, total_segs, g0, sc, lds, v, seg_out, reinterpret_cast<uint32_t*>(lds + LdsLayout<16>::kBytes + 1024), 512);
    } else {
      __shared__ uint32_t xch[kWaves16 / 2];
      slice_half<ChunkGeo, UnpackVisit<BLOCK, STAGE, NT>, CRC, 16, kWaves16>(geo, total_segs, g0, sc, lds, v, seg_out, xch,
                                                                         1);
    }
  }
}

// CRC only, one segment per wave.
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
crc32c_segments_once_kernel(const ChunkGeo geo, int64_t total_segs, const uint32_t* __restrict__ sc,
                            uint32_t* __restrict__ seg_out) {
  __shared__ uint4 lds_raw[kLdsBytes / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  NoVisit v;
  slice_once<ChunkGeo, NoVisit, true>(geo, total_segs, sc, lds, v, seg_out);
}

// store = 2: the same CRC walk on half of the waves (0-7) while the other half
// (8-15) stream the same segments' q bytes through the plain unpack (8 B of
// fp8 in, 16 B of bf16 out per lane: every load and store instruction fully
// coalesced), one segment behind or ahead, so the packed bytes come twice from
// L2 / the Infinity Cache instead of twice from HBM. In the fused walk every
// wave does both jobs in sequence: its CRC (LDS lookups, VALU) and its stores
// do not overlap, and the kernel takes about the sum of a CRC pass and an
// unpack pass (profiles/r3_kernels).
template <int BLOCK>
__device__ __forceinline__ void unpack_walk(const ChunkGeo& geo, int64_t total_segs, int64_t out_chunk_elems,
                                            uint16_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = __builtin_amdgcn_readfirstlane(int(blockIdx.x * 8 + ((threadIdx.x >> 6) & 7)));
  const int64_t nwaves = int64_t(gridDim.x) * 8;
  for (int64_t g = wave; g < total_segs; g += nwaves) {
    const Seg sg = geo(g);
    const int64_t n_q = sg.chunk_len / (BLOCK + 4) * BLOCK;
    if (sg.seg_start >= n_q) continue;  // the chunk's scales: nothing to unpack
    const float* scales = reinterpret_cast<const float*>(geo.src + sg.chunk_start + n_q);
    uint16_t* obase = out + sg.chunk * out_chunk_elems;
    const int64_t end = min(sg.seg_start + sg.len, n_q);
    const uint2* q = reinterpret_cast<const uint2*>(sg.p);
    constexpr int kU = 8;  // 8 x 512 B of loads in flight per wave
    for (int64_t base = 0; sg.seg_start + base < end; base += kU * 512) {
      uint2 v[kU];
      float sc[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t e = sg.seg_start + base + u * 512 + 8 * lane;
        v[u] = e < end ? q[(base + u * 512) / 8 + lane] : make_uint2(0, 0);
        sc[u] = e < end ? scales[e / BLOCK] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t e = sg.seg_start + base + u * 512 + 8 * lane;
        if (e >= end) continue;
        const float s = sc[u];
        *reinterpret_cast<uint4*>(obase + e) =
            make_uint4(fp8x2_to_bf16x2<false>(v[u].x, s), fp8x2_to_bf16x2<true>(v[u].x, s),
                       fp8x2_to_bf16x2<false>(v[u].y, s), fp8x2_to_bf16x2<true>(v[u].y, s));
      }
    }
  }
}

template <int BLOCK>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
verify_unpack_split_kernel(const ChunkGeo geo, int64_t total_segs, int64_t out_chunk_elems,
                           const uint32_t* __restrict__ sc, uint32_t* __restrict__ seg_out,
                           uint16_t* __restrict__ out) {
  __shared__ uint4 lds_raw[kLdsBytes / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  load_lds(lds, sc);
  if ((threadIdx.x >> 6) < 8) {
    const Slice4 st(lds);
    NoVisit v;
    slice_walk(geo, total_segs, sc, st, v, seg_out, 8);
  } else {
    unpack_walk<BLOCK>(geo, total_segs, out_chunk_elems, out);
  }
}

// A chunk's raw CRC: the XOR of its segments' values (each already shifted
// to the chunk end). Called by every thread of a kFoldThreads block; returns
// the raw CRC on thread 0.
// The loads go out four at a time (independent accumulators): a plain strided
// loop waits for each before the next (~9 round trips per 2112-segment chunk
// on 256 threads). A fold launch costs ~4.5 us whatever its work
// (profiles/r4_nt): folding in the fused kernel's last workgroup instead
// (generation-tagged slots that one workgroup polls) measured slower at
// 512 MiB, 159.8 vs 148.3 + 4.5 us, since one workgroup reads the slots at a
// fraction of the chip's rate (profiles/r4_fold_in_kernel).
constexpr int kFoldThreads = 1024;
__device__ uint32_t xor_chunk(const uint32_t* __restrict__ seg, int64_t nseg) {
  __shared__ uint32_t part[kFoldThreads / 64];
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  int64_t k = threadIdx.x;
  for (; k + 3 * kFoldThreads < nseg; k += 4 * kFoldThreads) {
    r0 ^= seg[k];
    r1 ^= seg[k + kFoldThreads];
    r2 ^= seg[k + 2 * kFoldThreads];
    r3 ^= seg[k + 3 * kFoldThreads];
  }
  for (; k < nseg; k += kFoldThreads) r0 ^= seg[k];
  uint32_t r = wave_xor_dpp(r0 ^ r1 ^ r2 ^ r3);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = r;
  __syncthreads();
  if (threadIdx.x != 0) return 0;
  r = 0;
#pragma unroll
  for (int i = 0; i < kFoldThreads / 64; ++i) r ^= part[i];
  return r;
}

// Per chunk: (x^(8*rem), init/xorout term) of full chunks [0..1] and of the short last chunk [2..3].
struct FoldTail {
  uint32_t xrem_full, init_full, xrem_last, init_last;
};

// One block per chunk.
__global__ void __launch_bounds__(kFoldThreads) crc32c_fold_kernel(const uint32_t* __restrict__ seg_out, int64_t bytes,
                                                                   int64_t chunk_bytes, int64_t spc, FoldTail t,
                                                                   uint32_t* __restrict__ out) {
  const int64_t c = blockIdx.x;
  const int64_t chunk_len = min(chunk_bytes, bytes - c * chunk_bytes);
  const bool full = chunk_len == chunk_bytes;
  const uint32_t r = xor_chunk(seg_out + c * spc, (chunk_len + kSegBytes - 1) / kSegBytes);
  if (threadIdx.x == 0) out[c] = r ^ (full ? t.init_full : t.init_last);
}

FoldTail fold_tail(int64_t chunk_bytes, int64_t last_len) {
  auto xrem = [](int64_t len) { return crc32c_xpow8n(uint64_t(len % kSegBytes)); };
  return FoldTail{xrem(chunk_bytes), crc32c_init_term(uint64_t(chunk_bytes)), xrem(last_len),
                  crc32c_init_term(uint64_t(last_len))};
}

// ---- batched: up to kCrcBatchMax independent buffers (the chunks one P2P
// group landed) in one segments launch + one fold launch.
struct BatchArgs {
  int n;
  int64_t seg_base[kCrcBatchMax + 1];  // prefix sums of the items' segment counts
  const uint8_t* src[kCrcBatchMax];
  int64_t bytes[kCrcBatchMax];
  uint32_t xrem[kCrcBatchMax];  // x^(8 * (bytes mod 16 KiB))
  uint32_t init[kCrcBatchMax];
  uint32_t* out[kCrcBatchMax];
};

__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
crc32c_batch_segments_kernel(const BatchArgs a, const uint32_t* __restrict__ sc, uint32_t* __restrict__ seg_out) {
  __shared__ uint4 lds_raw[kLdsBytes / 16];
  uint8_t* lds = reinterpret_cast<uint8_t*>(lds_raw);
  load_lds(lds, sc);
  const Slice4 st(lds);
  auto geo = [&](int64_t g) {
    int j = 0;
    while (g >= a.seg_base[j + 1]) ++j;
    const int64_t k = g - a.seg_base[j];
    Seg s;
    s.chunk = j;
    s.chunk_start = 0;
    s.chunk_len = a.bytes[j];
    s.seg_start = k * kSegBytes;
    s.p = a.src[j] + s.seg_start;
    s.len = min(int64_t(kSegBytes), a.bytes[j] - s.seg_start);
    s.xrem = a.xrem[j];
    return s;
  };
  NoVisit v;
  slice_walk(geo, a.seg_base[a.n], sc, st, v, seg_out);
}

__global__ void __launch_bounds__(kFoldThreads) crc32c_batch_fold_kernel(const BatchArgs a,
                                                                         const uint32_t* __restrict__ seg_out) {
  const int j = blockIdx.x;
  const uint32_t r = xor_chunk(seg_out + a.seg_base[j], a.seg_base[j + 1] - a.seg_base[j]);
  if (threadIdx.x == 0) *a.out[j] = r ^ a.init[j];
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
  for (int m = 0; m < 1024; ++m) h[size_t(kPow + m)] = crc32c_xpow8n(uint64_t(16) * uint64_t(m));
  for (int l = 0; l < 64; ++l) h[size_t(kLanePow + l)] = crc32c_xpow8n(uint64_t(kPieceBytes) * uint64_t(63 - l));
  const uint32_t xs = crc32c_xpow8n(kSegBytes);
  h[size_t(kSegPow)] = 0x80000000u;  // x^0
  for (int j = 1; j < kMaxSegs; ++j) h[size_t(kSegPow + j)] = crc32c_multmodp(xs, h[size_t(kSegPow + j - 1)]);
  const ConstEntry e = upload_consts(h, s);
  if (!e.d) return nullptr;
  g_consts.by_device[dev] = e;
  return e.d;
}

// One workgroup per CU (LDS-bound), 16 segments per workgroup at a time,
// grid-stride beyond that. Kernel trace on 1 GiB (profiles/r2_crc_slice):
// 186.5 us with 256 workgroups, 185.0 with 512, 187.8 with 1024.
// Workgroups for a segment walk: as few rounds of kWaves segments per
// workgroup as `cap` allows, then as few workgroups as still need only that
// many rounds. A wave takes segments g, g + nwaves, ..., so a last round that
// only some waves reach costs a whole round: 16896 segments (512 MiB of
// bf16 packed) on 256 x 16 waves are 4.125 rounds, 5 for the kernel; 212
// workgroups do the same 5 rounds with every wave busy, and the freed CUs'
// share of HBM goes to the rest: fused verify+unpack 4.30 -> 4.61 TB/s
// (profiles/r3_tail).
dim3 seg_grid(int64_t total_segs, int max_blocks) {
  const int64_t cap = max_blocks > 0 ? max_blocks : 256;
  const int64_t rounds = std::max<int64_t>(1, (total_segs + cap * kWaves - 1) / (cap * kWaves));
  const int64_t blocks = (total_segs + kWaves * rounds - 1) / (kWaves * rounds);
  return dim3(unsigned(std::max<int64_t>(1, std::min<int64_t>(blocks, cap))));
}

// Resident once16 workgroups on the device (per CU x CUs), cached per device.
int once16_slots() {
  static std::mutex mu;
  static std::map<int, int> by_device;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  if (auto it = by_device.find(dev); it != by_device.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, verify_unpack_once16_kernel<128>, kWaves16 * 64, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 512;
  return by_device[dev] = std::max(1, per_cu) * std::max(1, cus);
}

// Grid of the one-segment-per-wave kernel with its last, partial round of
// workgroups done in half segments (slice_half). Every workgroup lasts about
// as long, so with W workgroups on S slots the kernel takes ceil(W / S)
// rounds even when the last holds only a few: 16896 segments (512 MiB of bf16
// packed) are 2112 workgroups on 512 slots, 4.125 rounds. Cutting the last
// round's segments in halves gives twice the workgroups at half the length,
// so a last round up to half full ends in half the time. W <= S / 2: every
// segment in halves (twice the parallelism); otherwise no split.
struct OnceGrid {
  int64_t split_block;  // workgroups [0, split_block) take whole segments
  unsigned blocks;
};
OnceGrid once_split(int64_t total_segs, bool split) {
  const int64_t W = (total_segs + kWaves16 - 1) / kWaves16, S = once16_slots();
  int64_t full = W;
  if (split) {
    if (W <= S) full = 2 * W <= S ? 0 : W;
    else if (const int64_t tail = W % S; tail && 2 * tail <= S) full = W - tail;
  }
  const int64_t half_segs = std::max<int64_t>(0, total_segs - full * kWaves16);
  return OnceGrid{full, unsigned(full + (half_segs + kWaves16 / 2 - 1) / (kWaves16 / 2))};
}

struct Plan {
  int64_t spc, nchunks, total_segs;
  uint32_t* consts;
  FoldTail tail;
};

hipError_t plan(int64_t bytes, int64_t chunk_bytes, Plan* p, hipStream_t s) {
  p->spc = (chunk_bytes + kSegBytes - 1) / kSegBytes;
  if (p->spc > kMaxSegs) return hipErrorInvalidValue;  // chunks up to 1 GiB (segpow table)
  p->nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  const int64_t last_len = bytes - (p->nchunks - 1) * chunk_bytes;
  p->total_segs = (p->nchunks - 1) * p->spc + (last_len + kSegBytes - 1) / kSegBytes;
  p->consts = device_consts(s);
  p->tail = fold_tail(chunk_bytes, last_len);
  return p->consts ? hipSuccess : hipErrorOutOfMemory;
}

}  // namespace

hipError_t crc32c_warm(int64_t chunk_bytes, hipStream_t s) {
  if ((chunk_bytes + kSegBytes - 1) / kSegBytes > kMaxSegs) return hipErrorInvalidValue;
  return device_consts(s) ? hipSuccess : hipErrorOutOfMemory;
}

size_t crc32c_workspace_bytes(int64_t bytes, int64_t chunk_bytes) {
  if (bytes <= 0 || chunk_bytes <= 0) return 16;
  int64_t spc = (chunk_bytes + kSegBytes - 1) / kSegBytes;
  int64_t nchunks = (bytes + chunk_bytes - 1) / chunk_bytes;
  return size_t(nchunks * spc * 4 + 16);
}

hipError_t crc32c_chunks(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                         hipStream_t s) {
  return crc32c_chunks_capped(src, bytes, chunk_bytes, out, workspace, s, 0);
}

hipError_t crc32c_chunks_capped(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                                hipStream_t s, int max_blocks) {
  if (bytes <= 0) return hipSuccess;
  if (chunk_bytes <= 0 || (reinterpret_cast<uintptr_t>(src) & 15)) return hipErrorInvalidValue;
  // One chunk (the engine's per-chunk checks) may have any length: only a
  // chunk's last segment is partial, and it takes a byte tail. Several chunks
  // need a 16-B multiple so that every chunk starts 16-B aligned.
  if (bytes <= chunk_bytes) chunk_bytes = bytes;
  else if (chunk_bytes % 16) return hipErrorInvalidValue;
  Plan p;
  if (hipError_t e = plan(bytes, chunk_bytes, &p, s); e != hipSuccess) return e;
  auto* seg = static_cast<uint32_t*>(workspace);
  const ChunkGeo geo{static_cast<const uint8_t*>(src), bytes, chunk_bytes, p.spc, p.tail.xrem_full, p.tail.xrem_last};
  crc32c_segments_kernel<<<seg_grid(p.total_segs, max_blocks), dim3(kThreads), 0, s>>>(geo, p.total_segs, p.consts,
                                                                                        seg);
  crc32c_fold_kernel<<<dim3(unsigned(p.nchunks)), dim3(kFoldThreads), 0, s>>>(seg, bytes, chunk_bytes, p.spc, p.tail,
                                                                              out);
  return hipGetLastError();
}

size_t crc32c_batch_workspace_bytes(int64_t max_item_bytes, int n) {
  const int64_t spc = (std::max<int64_t>(max_item_bytes, 1) + kSegBytes - 1) / kSegBytes;
  return size_t(int64_t(std::max(n, 1)) * spc * 4 + 16);
}

hipError_t crc32c_batch(const CrcItem* items, int n, void* workspace, hipStream_t s, int max_blocks) {
  if (n <= 0) return hipSuccess;
  if (n > kCrcBatchMax) return hipErrorInvalidValue;
  BatchArgs a{};
  a.n = 0;
  a.seg_base[0] = 0;
  uint32_t* consts = device_consts(s);
  if (!consts) return hipErrorOutOfMemory;
  for (int i = 0; i < n; ++i) {
    const CrcItem& it = items[i];
    if (it.bytes <= 0) continue;
    if (reinterpret_cast<uintptr_t>(it.src) & 15) return hipErrorInvalidValue;  // any length
    const int64_t spc = (it.bytes + kSegBytes - 1) / kSegBytes;
    if (spc > kMaxSegs) return hipErrorInvalidValue;
    const int j = a.n++;
    a.src[j] = static_cast<const uint8_t*>(it.src);
    a.bytes[j] = it.bytes;
    a.xrem[j] = crc32c_xpow8n(uint64_t(it.bytes % kSegBytes));
    a.init[j] = crc32c_init_term(uint64_t(it.bytes));
    a.out[j] = it.out;
    a.seg_base[j + 1] = a.seg_base[j] + spc;
  }
  if (a.n == 0) return hipSuccess;
  auto* seg = static_cast<uint32_t*>(workspace);
  crc32c_batch_segments_kernel<<<seg_grid(a.seg_base[a.n], max_blocks), dim3(kThreads), 0, s>>>(a, consts, seg);
  crc32c_batch_fold_kernel<<<dim3(unsigned(a.n)), dim3(kFoldThreads), 0, s>>>(a, seg);
  return hipGetLastError();
}

hipError_t fp8_verify_unpack(const void* packed, int64_t src_bytes, int64_t src_chunk, int block, uint16_t* out,
                             uint32_t* crc_out, void* workspace, hipStream_t s, int max_blocks, int store) {
  if (src_bytes <= 0) return hipSuccess;
  if (src_chunk <= 0 || src_chunk % 4096 || src_bytes % (2 * block) || (reinterpret_cast<uintptr_t>(packed) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 15))
    return hipErrorInvalidValue;
  const int64_t pchunk = src_chunk / 2 + src_chunk / 2 / block * 4;
  const int64_t full = src_bytes / src_chunk, tail = src_bytes % src_chunk;
  const int64_t bytes = full * pchunk + (tail ? tail / 2 + tail / 2 / block * 4 : 0);
  Plan p;
  if (hipError_t e = plan(bytes, pchunk, &p, s); e != hipSuccess) return e;
  auto* seg = static_cast<uint32_t*>(workspace);
  const ChunkGeo geo{static_cast<const uint8_t*>(packed), bytes, pchunk, p.spc, p.tail.xrem_full, p.tail.xrem_last};
  const int64_t oc = src_chunk / 2;
  const dim3 grid = seg_grid(p.total_segs, max_blocks), tpb{kThreads};
  if (store < 0) store = kFusedStoreDefault;
  // the split kernel's CRC half walks 8 segments per workgroup at a time
  const dim3 grid2(unsigned(std::max<int64_t>(1, std::min<int64_t>((p.total_segs + 7) / 8, max_blocks > 0 ? max_blocks : 256))));
  const dim3 grid5(unsigned((p.total_segs + kWaves - 1) / kWaves));  // store 5: one segment per wave
  const OnceGrid og = once_split(p.total_segs, store != 10);
  const dim3 grid7(og.blocks), tpb7(kWaves16 * 64);
  const int64_t sb = og.split_block;
#define DLD_VU(B)                                                                                           \
  (store == 9   ? (verify_unpack_once16_kernel<B, true, false><<<grid7, tpb7, 0, s>>>(geo, p.total_segs, sb, oc, p.consts, seg, out)) \
   : store == 14 ? (verify_unpack_once16_kernel<B, true, false, true><<<grid7, tpb7, 0, s>>>(geo, p.total_segs, sb, oc, p.consts, seg, out)) \
   : store == 13 ? (verify_unpack_once16_kernel<B, true, true, false><<<grid7, tpb7, 0, s>>>(geo, p.total_segs, sb, oc, p.consts, seg, out)) \
   : store == 7 || store == 10 ? (verify_unpack_once16_kernel<B, true, true, true><<<grid7, tpb7, 0, s>>>(geo, p.total_segs, sb, oc, p.consts, seg, out))  \
   : store == 5 ? (verify_unpack_once_kernel<B><<<grid5, tpb, 0, s>>>(geo, p.total_segs, oc, p.consts, seg, out))      \
   : store == 2 ? (verify_unpack_split_kernel<B><<<grid2, tpb, 0, s>>>(geo, p.total_segs, oc, p.consts, seg, out))     \
   : store == 1 ? (verify_unpack_segments_kernel<B, true><<<grid, tpb, 0, s>>>(geo, p.total_segs, oc, p.consts, seg, out)) \
                : (verify_unpack_segments_kernel<B, false><<<grid, tpb, 0, s>>>(geo, p.total_segs, oc, p.consts, seg, out)))
  if (store == 8) {  // diagnostic: store 7 without the CRC math
    if (block != 128) return hipErrorInvalidValue;
    verify_unpack_once16_kernel<128, false, true, true><<<grid7, tpb7, 0, s>>>(geo, p.total_segs, sb, oc, p.consts, seg, out);
  } else if (store == 3 || store == 4 || store == 6) {  // diagnostic: the same walk without the CRC math (CRCs are garbage)
    if (block != 128) return hipErrorInvalidValue;
    if (store == 3)
      verify_unpack_segments_kernel<128, true, false><<<grid, tpb, 0, s>>>(geo, p.total_segs, oc, p.consts, seg, out);
    else if (store == 4)
      verify_unpack_segments_kernel<128, false, false><<<grid, tpb, 0, s>>>(geo, p.total_segs, oc, p.consts, seg, out);
    else
      verify_unpack_once_kernel<128, false><<<grid5, tpb, 0, s>>>(geo, p.total_segs, oc, p.consts, seg, out);
  } else {
    switch (block) {
      case 32: DLD_VU(32); break;
      case 64: DLD_VU(64); break;
      case 128: DLD_VU(128); break;
      case 256: DLD_VU(256); break;
      case 512: DLD_VU(512); break;
      default: return hipErrorInvalidValue;
    }
  }
#undef DLD_VU
  crc32c_fold_kernel<<<dim3(unsigned(p.nchunks)), dim3(kFoldThreads), 0, s>>>(seg, bytes, pchunk, p.spc, p.tail,
                                                                              crc_out);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace dissem
