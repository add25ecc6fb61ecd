// MI355X backend of the planned engine: HBM slots (hipMalloc), RCCL grouped
// point-to-point over xGMI on one communicator + stream per comm lane,
// hipMemcpyAsync staging from pinned host memory (one or two copy streams), and
// the gfx950 CRC32C kernel (verify stream).
//
// Hardware queues: HIP maps ordinary streams onto a pool of GPU_MAX_HW_QUEUES
// (4) queues, so streams can share one; a CU-masked stream always gets a queue
// of its own. With peers the verify stream is masked to the last verify_cus
// CUs and every comm lane and copy stream to the others (verify_cus below), so
// no RCCL kernel waiting for a peer can hold back a copy, a check or another
// lane (queue ids: profiles/r2_queues/ at 3 ranks, profiles/r2_queues8/ at 8
// ranks with 14 lanes each) and no CRC workgroup shares a CU with RCCL.
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>

#include "engine/backend.h"
#include "engine/planned_engine.h"

namespace dissem {

struct HipBackendConfig {
  int device = 0;
  int rank = 0;
  int world = 1;
  std::string nccl_uid;  // ncclUniqueId bytes (world > 1): one id, or one per lane (parallel init)
  int64_t max_chunk_bytes = 64ll << 20;  // largest source chunk staged (sizes the fp8 packing scratch)
  // world == 1: still build a one-rank communicator, so P2P groups to self
  // exercise the RCCL path on a single-GPU box (rccl_selftest)
  bool self_comm = false;
  // > 0: the verify and copy streams get a CU mask that leaves this many CUs
  // free for the comm stream's RCCL kernels (hipExtStreamCreateWithCUMask).
  int reserve_cus = 0;
  // > 0: the verify stream runs on the LAST verify_cus CU-mask bits only and
  // every comm lane and copy stream on the others, so no CRC workgroup shares a
  // CU with an RCCL kernel. Mask bit i is CU i / 8 of XCD i mod 8 (bin/contention
  // -cumap), so the last 32 bits are 4 CUs on each of the 8 XCDs: keep
  // verify_cus a multiple of 8 (an XCD left with no CU ignores its mask).
  // bin/contention -paced (profiles/r4_contention/paced_partitioned.jsonl): a
  // 64-workgroup copy keeps 99.6 % of its alone rate beside 450 GB/s of
  // continuous verification on the last 32 bits, against 93.8 % beside an
  // unmasked full-grid verify and 85.6 % beside a 32-workgroup one. Overrides
  // reserve_cus; the verify kernels size their grid's last round for verify_cus.
  int verify_cus = 0;
  int nccl_min_ctas = 0, nccl_max_ctas = 0;  // 0: RCCL default
  int lanes = 1;                               // comm lanes (communicator + stream each)
  int hosts = 1;                               // multi-node: hosts of world / hosts ranks (backend.h host_lanes)
  int host_lane_classes = 0;
  bool nccl_register = false;                  // ncclCommRegister every layer slot
  bool parallel_init = true;                   // per-lane ids: init all lane communicators in one group
};

// A non-default stream whose kernels may use every CU but the last `reserve`
// (reserve <= 0: a plain non-blocking stream, or with `dedicated` a stream
// masked to every CU, which gets a hardware queue of its own).
hipStream_t create_stream_reserving(int device, int reserve, bool dedicated = false);
// A stream whose kernels run on the last `cus` CU-mask bits only.
hipStream_t create_stream_on_last(int device, int cus);

std::unique_ptr<Backend> make_hip_backend(const HipBackendConfig& cfg);
std::shared_ptr<HostBuffer> alloc_pinned(int64_t size);
std::string nccl_unique_id(int count = 1);  // `count` ncclUniqueIds, concatenated

}  // namespace dissem
