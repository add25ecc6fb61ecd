// Launchers for the gfx950 kernels. Callable from host C++ (g++ objects); the
// kernels themselves are in csrc/kernels/*.hip, compiled for gfx950 only.
//
// All of them are single-pass streaming kernels: every input byte is read once
// and every output byte written once, 16 B per lane, with no data shared
// between workgroups. The hardware's round-robin of workgroups over the 8 XCDs
// therefore needs no remapping (there is no L2 reuse to keep on one XCD); what
// matters is enough bytes in flight per CU (HBM latency) and, for CRC32C, the
// LDS table layout (crc32c.hip). fill sizes its grid to the CU count (256)
// times the workgroups a CU holds and grid-strides beyond that; the CRC32C
// grids are described below; fp8 pack/unpack give every lane one 8-element
// group (a 64 MiB chunk is 16k workgroups, far more than the chip holds at once).
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

// ---- crc32c.hip: CRC32C verification (and the fused fp8 unpack) on gfx950.
// Two kernels: the CRC-only check walks (one 1024-thread workgroup per CU,
// each a contiguous range of 16 KiB segments), the fused check + unpack runs
// one segment per wave (512-thread workgroups, two per CU). Both fold a
// chunk's segments inside the same launch (device-scope atomics on one 64-bit
// {acc, count} word per item in `workspace`, 8-B aligned; crc32c.hip). A workspace must be
// zeroed ONCE (e.g. hipMemsetAsync) before its first use; every launch leaves
// it zeroed again. Launches that share a workspace must be ordered (one stream).
// `cus`: the CUs the launch's stream may use (a CU-masked verify stream): the
// walk launches one workgroup per such CU, the fused kernel sizes its grid's
// last partial round for them. 0 = the whole device.
//
// out[c] (device or host-mapped memory) receives the standard CRC32C of chunk
// c of [src, src+bytes). src 16-B aligned; chunk_bytes a multiple of 16
// unless the span is one chunk (bytes <= chunk_bytes: any length).
size_t crc32c_workspace_bytes(int64_t bytes, int64_t chunk_bytes);
// Upload the CRC tables (stream-ordered on s) ahead of time; later launches
// then never allocate or copy. Never a host-synchronous copy.
hipError_t crc32c_warm(hipStream_t s);
hipError_t crc32c_chunks(const void* src, int64_t bytes, int64_t chunk_bytes, uint32_t* out, void* workspace,
                         hipStream_t s, int cus = 0);
// Batched: the standard CRC32C of each of up to kCrcBatchMax independent
// buffers (any length, 16-B aligned) in one launch - the chunks one P2P group
// or one staging batch landed. `workspace`: crc32c_batch_workspace_bytes().
constexpr int kCrcBatchMax = 16;
struct CrcItem {
  const void* src;
  int64_t bytes;
  uint32_t* out;
};
size_t crc32c_batch_workspace_bytes();
hipError_t crc32c_batch(const CrcItem* items, int n, void* workspace, hipStream_t s, int cus = 0);

// ---- fp8.hip: bf16 -> OCP fp8 e4m3fn with one f32 scale per `block` elements
// (power-of-two scale 2^E, core/fp8.h; +-inf saturate, NaN stays NaN), and back.
hipError_t fp8_pack(const uint16_t* bf16, int64_t n, uint8_t* fp8, float* scales, int block, hipStream_t s);
hipError_t fp8_unpack(const uint8_t* fp8, const float* scales, int64_t n, uint16_t* bf16, int block, hipStream_t s);
// Whole layer into the chunked packed layout of core/fp8.h (one pack launch per chunk).
hipError_t fp8_pack_chunks(const void* src, int64_t src_bytes, int64_t src_chunk, int block, void* dst,
                           hipStream_t s);

// ---- crc32c.hip: fused verify + unpack of a packed layer: crc_out[c] = CRC32C of
// packed chunk c, out = the bf16 layer (src_bytes). One pass over the packed bytes.
// `workspace`: crc32c_workspace_bytes(packed bytes, packed chunk) bytes, zeroed once.
hipError_t fp8_verify_unpack(const void* packed, int64_t src_bytes, int64_t src_chunk, int block, uint16_t* out,
                             uint32_t* crc_out, void* workspace, hipStream_t s, int cus = 0);
// Batched: up to kCrcBatchMax independent packed chunks (each the core/fp8.h
// image of `src_len` bf16 source bytes) in one launch: CRC32C of each packed
// chunk to *crc_out, its bf16 values to out. `workspace`: crc32c_batch_workspace_bytes().
struct FusedItem {
  const void* packed;
  int64_t src_len;
  uint16_t* out;
  uint32_t* crc_out;
};
hipError_t fp8_verify_unpack_batch(const FusedItem* items, int n, int block, void* workspace, hipStream_t s,
                                   int cus = 0);

}  // namespace kern
}  // namespace dissem
