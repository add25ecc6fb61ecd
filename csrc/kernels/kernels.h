// Launchers for the gfx950 kernels. Callable from host C++ (g++ objects); the
// kernels themselves are in csrc/kernels/*.hip, compiled for gfx950 only.
//
// All of them are single-pass streaming kernels: every input byte is read once
// and every output byte written once, 16 B per lane, with no data shared
// between workgroups. The hardware's round-robin of workgroups over the 8 XCDs
// therefore needs no remapping (there is no L2 reuse to keep on one XCD); what
// matters is enough bytes in flight per CU (HBM latency) and, for CRC32C, the
// LDS table layout (crc32c.hip). fill and CRC32C size their grids to the CU
// count (256) times the workgroups a CU holds and grid-stride beyond that;
// fp8 pack/unpack give every lane one 8-element group (a 64 MiB chunk is
// 16k workgroups, far more than the chip holds at once).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace dissem {
namespace kern {

// ---- fill.hip: counter-based random bytes (splitmix64 of (seed, u64 index)),
// 16 B per lane stores; byte-identical to kern::fill_random_host.
hipError_t fill_random(void* dst, int64_t bytes, uint64_t seed, hipStream_t s);
void fill_random_host(void* dst, int64_t bytes, uint64_t seed, int64_t offset = 0);
// Test helper: hold stream s until *flag != 0 (host-mapped) or max_iters ~3 us sleeps.
hipError_t spin_until(const uint32_t* flag, uint64_t max_iters, uint64_t* iters, hipStream_t s);
// Read-bandwidth probe: XOR of [src, src+bytes) into blocks*4 dwords at out
// (bytes % 16 == 0); `depth` 16-B loads in flight per lane (1, 2, 4, 8).
hipError_t read_xor(const void* src, int64_t bytes, uint32_t* out, int blocks, int depth, hipStream_t s);
// Segment-read probe (the CRC kernels' load shape, no compute): 16 KiB per
// wave, 1024-thread workgroups, `blocks` of them; layout 0 = 64-B lane pieces,
// 1 = strided 16-B words; roll = prefetch the next segment while consuming.
// out: blocks * 1024 dwords; bytes % 16384 == 0.
hipError_t read_seg(const void* src, int64_t bytes, uint32_t* out, int blocks, int layout, bool roll, hipStream_t s);

// ---- crc32c.hip: CRC32C of every `chunk_bytes` chunk of [src, src+bytes).
// out[c] (device or host-mapped memory) receives the standard CRC32C of chunk c.
// `workspace` must hold crc32c_workspace_bytes(bytes, chunk_bytes) bytes of
// device memory. src 16-B aligned; chunk_bytes a multiple of 16 unless the span
// is one chunk (bytes <= chunk_bytes: any length, e.g. a layer's last chunk).
size_t crc32c_workspace_bytes(int64_t bytes, int64_t chunk_bytes);
// Build and upload (stream-ordered on s) the CRC tables and the fold tables of
// `chunk_bytes` chunks ahead of time; later launches then never allocate. Any
// table first needed later is uploaded the same way, never with a host sync.
hipError_t crc32c_warm(int64_t chunk_bytes, hipStream_t s);
hipError_t crc32c_chunks(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                         hipStream_t s);
// Batched: the standard CRC32C of each of up to kCrcBatchMax independent
// buffers (any length, 16-B aligned) in one launch pair - the chunks a P2P
// group landed. `workspace`: crc32c_batch_workspace_bytes(max bytes, n).
constexpr int kCrcBatchMax = 16;
struct CrcItem {
  const void* src;
  int64_t bytes;
  uint32_t* out;
};
size_t crc32c_batch_workspace_bytes(int64_t max_item_bytes, int n);
// crc32c_chunks with the segment kernel's grid capped at max_blocks workgroups
// (0 = one per CU); capped grids put many segments on every wave (tests, A/B).
// The segment kernel (slice-by-4 byte tables on lane-contiguous 64-B pieces of
// coalesced loads) and the variants it replaced: crc32c.hip, profiles/r2_crc_ab.
hipError_t crc32c_chunks_capped(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                                hipStream_t s, int max_blocks);
// max_blocks (here and in fp8_verify_unpack): cap on the segment kernel's grid,
// one workgroup per CU (0 = all 256); a CU-masked stream passes its CU count so
// no workgroup waits for a second wave.
hipError_t crc32c_batch(const CrcItem* items, int n, void* workspace, hipStream_t s, int max_blocks = 0);

// ---- fp8.hip: bf16 -> OCP fp8 e4m3fn with one f32 scale per `block` elements
// (power-of-two scale 2^E, core/fp8.h; +-inf saturate, NaN stays NaN), and back.
hipError_t fp8_pack(const uint16_t* bf16, int64_t n, uint8_t* fp8, float* scales, int block, hipStream_t s);
hipError_t fp8_unpack(const uint8_t* fp8, const float* scales, int64_t n, uint16_t* bf16, int block, hipStream_t s);
// Whole layer into the chunked packed layout of core/fp8.h (one pack launch per chunk).
hipError_t fp8_pack_chunks(const void* src, int64_t src_bytes, int64_t src_chunk, int block, void* dst,
                           hipStream_t s);

// ---- crc32c.hip: fused verify + unpack of a packed layer: crc_out[c] = CRC32C of
// packed chunk c, out = the bf16 layer (src_bytes). One pass over the packed bytes.
// `workspace`: crc32c_workspace_bytes(packed bytes, packed chunk) bytes.
// store: how the bf16 output leaves the CU - 0 = each lane's 32 B straight from
// registers (two half-dense 2 KiB stores per word), 1 = through 1 KiB of LDS per
// wave as fully coalesced 1 KiB stores, 2 = split roles: half of each
// workgroup's waves CRC the segments while the other half unpack them;
// 5 = one segment per wave (1024-thread workgroups, 32 table replicas), 7 = the
// same with 512-thread workgroups and 16 replicas (two per CU), the grid's
// last partial round in half segments and nontemporal staged stores, 9 = 7
// with direct stores (temporal), 10 = 7 without the half-segment round, 13 = 7
// with temporal stores, 14 = 9 with nontemporal ones; 3, 4, 6, 8 are no-CRC
// diagnostics (their CRCs are garbage); -1 = kFusedStoreDefault.
// 7: 5.3-5.4 TB/s at 512 MiB, 5.9-6.2 at 4 GiB vs store 1's 4.66 / 4.89
// (profiles/r4_nt, profiles/r4_kernels_final)
constexpr int kFusedStoreDefault = 7;
hipError_t fp8_verify_unpack(const void* packed, int64_t src_bytes, int64_t src_chunk, int block, uint16_t* out,
                             uint32_t* crc_out, void* workspace, hipStream_t s, int max_blocks = 0, int store = -1);

}  // namespace kern
}  // namespace dissem
