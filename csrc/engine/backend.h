// Device backend of the planned data engine. The engine (csrc/engine/
// planned_engine.cc) owns scheduling: piece order, group formation, chunk
// states, verification bookkeeping. A backend owns the device: memory, the
// three ordered queues (comm, copy, verify) and completion events.
//
//  * HipBackend (csrc/gpu/hip_backend.cc): HBM via hipMalloc, RCCL grouped
//    P2P on one world communicator over xGMI, hipMemcpyAsync H2D staging,
//    the gfx950 CRC32C kernel, hipEvents.
//  * SimBackend (csrc/engine/sim_backend.cc): host memory, worker threads as
//    in-order queues, and an in-process "fabric" that matches sends and recvs
//    between ranks FIFO per (src, dst) exactly like RCCL P2P (a group blocks its
//    queue until every op in it is matched). Used to test multi-rank schedules,
//    including deadlock freedom, without GPUs.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace dissem {

using Ev = uint64_t;  // 0 = no event

struct XOp {
  bool send;
  int peer;  // partner rank; the root rank when bcast
  uint8_t* ptr;
  int64_t len;
  bool bcast = false;  // collective broadcast of [ptr, ptr+len) from rank `peer` to every rank (in place)
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  virtual void init_thread() {}  // called on the engine's issue thread
  virtual uint8_t* alloc(int64_t n) = 0;
  virtual void free(uint8_t* p) = 0;
  virtual void zero_sync(uint8_t* p, int64_t n) = 0;
  // page-aligned host staging memory the copy queue can DMA from (pinned on GPUs)
  virtual uint8_t* alloc_host(int64_t n) = 0;
  virtual void free_host(uint8_t* p) = 0;
  // copy queue: async host -> device copy; event fires when it landed
  virtual Ev stage(uint8_t* dst, const uint8_t* src_host, int64_t n) = 0;
  // copy queue: host -> device copy of `n_src` bytes of bf16, then fp8-pack them
  // into dst in the packed chunk layout of core/fp8.h
  virtual Ev stage_pack(uint8_t* dst, const uint8_t* src_host, int64_t n_src, int block) = 0;
  // comm queue: wait for `waits`, then one grouped set of P2P sends/recvs
  virtual Ev group(const std::vector<XOp>& ops, const std::vector<Ev>& waits) = 0;
  // comm queue (fault injection): overwrite 4 bytes at p behind everything
  // queued so far, e.g. a chunk a group just received
  virtual Ev corrupt(uint8_t* p) = 0;
  // verify queue: after `after`, CRC32C of [p, p+n) into result slot `slot`
  // (n == 0: just an ordering marker on the verify queue)
  virtual Ev crc(const uint8_t* p, int64_t n, uint32_t slot, Ev after) = 0;
  // verify queue: after `after`, CRC32C of several independent buffers (the
  // chunks one P2P group landed) into their result slots; one event for all.
  struct CrcReq {
    const uint8_t* p;
    int64_t n;
    uint32_t slot;
  };
  virtual Ev crc_batch(const std::vector<CrcReq>& reqs, Ev after) {
    Ev last = 0;
    for (auto& r : reqs) {
      if (last) release(last);
      last = crc(r.p, r.n, r.slot, after);
    }
    return last ? last : crc(nullptr, 0, 0, after);
  }
  virtual int query(Ev e) = 0;  // 1 done, 0 pending, -1 failed
  virtual void release(Ev e) = 0;
  virtual uint32_t crc_result(uint32_t slot) = 0;
  virtual std::string async_error() { return ""; }
  // Elastic recovery: abort every in-flight comm-queue operation, then continue
  // on a communicator of the surviving ranks (the same call on every survivor,
  // with the same `dead` ranks, `generation` and `comm_id`). Returns this
  // rank's new index. RCCL: ncclCommAbort, then ncclCommInitRank of the
  // survivors with the leader's fresh unique id (comm_id).
  virtual std::string new_comm_id() { return ""; }
  virtual int shrink(const std::vector<int>& dead, uint64_t generation, const std::string& comm_id) {
    (void)dead;
    (void)generation;
    (void)comm_id;
    throw std::runtime_error(name() + " backend cannot shrink its communicator");
  }
  virtual void sync_all() = 0;
  virtual void destroy(bool abort) = 0;
};

struct SimFabricStats {
  int64_t matched = 0, bytes = 0;
};

// In-process simulated fabric: ranks of one "communicator" share `comm_key`.
std::unique_ptr<Backend> make_sim_backend(const std::string& comm_key, int rank, int world);
SimFabricStats sim_fabric_stats(const std::string& comm_key);

}  // namespace dissem
