// MI355X data plane: RCCL point-to-point over xGMI + HBM store + host/NVMe
// staging + gfx950 CRC32C verification.
//
// Execution model (replaces the reference's "goroutine + fresh TCP connection
// per layer", transport.go:267-275):
//  * The leader turns every scheduling decision (mode 0/1/2/3) into XferJobs
//    with global sequence numbers and sends each rank its share (XferBatch).
//  * Each job is cut into chunk-sized pieces on a fixed grid. A rank orders its
//    pieces by (piece index, sequence number) - a key every rank computes the
//    same way - and issues them as ncclGroupStart/End batches on ONE world
//    communicator and ONE stream. A batch holds at most one send and one recv
//    per peer, so every group is an all-to-all round that keeps all 7 xGMI links
//    of a GPU busy. Because every rank posts its pieces in one global order,
//    the schedule cannot deadlock (proof sketch in gpu_engine.cc), no matter how
//    the leader interleaves jobs (mode 2 dispatches them dynamically).
//  * Host-tier sources are staged chunk by chunk with hipMemcpyAsync on a copy
//    stream; the comm stream waits on the chunk's event, so PCIe staging and
//    xGMI transfer pipeline per chunk (the reference's pipe/tee, at chunk grain).
//  * Every landed chunk is checksummed by the CRC32C kernel on a verify stream
//    against the holder's announced manifest before the node acks it.
// Streams: comm, copy, verify (+ torch's default) fit in 4 hardware queues.
#pragma once

#include <hip/hip_runtime_api.h>
#include <rccl.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine/engine.h"

namespace dissem {

struct GpuEngineConfig {
  int device = 0;
  int rank = 0;
  int world = 1;
  std::vector<NodeID> rank_nodes;  // rank -> node id
  std::string nccl_uid;            // ncclUniqueId bytes for the world communicator (world > 1)
  int64_t chunk_bytes = 64ll << 20;
  bool verify = true;
  bool poison = true;              // zero non-seeded slots between sessions
  int max_inflight_groups = 64;
  int group_peers = 0;             // ops per peer per group (0 = 1 send + 1 recv per peer)
};

struct GpuEngineStats {
  int64_t bytes_sent = 0, bytes_recv = 0, bytes_staged = 0, bytes_verified = 0;
  int64_t groups = 0, pieces = 0, verify_failures = 0, unverified_pieces = 0;
  double issue_ms = 0;  // host time spent enqueueing
};

class GpuEngine : public DataEngine {
 public:
  explicit GpuEngine(const GpuEngineConfig& cfg);
  ~GpuEngine() override;

  // ---- setup (call before a session; not thread-safe with a running session)
  uint8_t* provision(LayerID layer, int64_t size);
  uint8_t* device_ptr(LayerID layer);
  void set_manifest(LayerID layer, const CrcManifest& m);
  void set_seeded(LayerID layer, bool device_resident);
  void reset_session();  // wait idle, forget landed chunks, poison non-seeded slots
  GpuEngineStats stats();
  std::string error();

  // ---- DataEngine
  std::string name() const override { return "rccl"; }
  Location target() const override { return Location::Device; }
  bool planned() const override { return true; }
  int64_t chunk_bytes() const override { return cfg_.chunk_bytes; }
  std::map<LayerID, CrcManifest> manifest() override;
  bool on_message(const MessagePtr& m) override;
  void send_range(NodeID dest, LayerID layer, int64_t offset, int64_t size, int64_t total, int64_t rate) override;
  void load_range(LayerID layer, int64_t offset, int64_t size, int64_t total, int64_t rate) override;
  void quiesce() override;
  void shutdown() override;

  hipStream_t comm_stream() const { return comm_stream_; }
  int rank_of(NodeID n) const;

 private:
  enum class Kind : uint8_t { Send, Recv, Local };
  struct Piece {
    Kind kind;
    uint64_t seq;
    int64_t pidx;  // piece index inside its job (ordering key, major)
    int peer;      // rank
    LayerID layer;
    int64_t off, len, total;
    int64_t chunk;     // grid chunk index
    bool full;         // covers the whole grid chunk
    bool has_crc = false;
    uint32_t crc = 0;
    NodeID src_node;
  };
  struct Layer {
    int64_t size = 0;
    uint8_t* dev = nullptr;
    bool seeded = false;
    CrcManifest manifest;
    std::vector<uint8_t> st;        // per chunk: 0 absent, 1 pending, 2 resident
    std::vector<hipEvent_t> ev;     // event that makes a pending chunk valid
    std::vector<uint8_t> on_comm;   // pending event was recorded on the comm stream
    std::vector<uint8_t> want;      // inject Landed when resident (assigned to this rank)
  };
  struct Verify {  // outstanding landing (recv group or staging copy) awaiting its CRC check
    hipEvent_t ev;
    std::vector<Piece> pieces;
    std::vector<uint32_t> slots;  // CRC result slots (pinned), ~0u = not verified
  };
  struct Req {
    enum Type { Batch, Load, Reset, Quiesce, Stop } type;
    std::vector<XferJob> jobs;
    LayerID layer = 0;
    int64_t off = 0, len = 0;
  };

  void run();
  void take_requests(bool block);
  void add_batch(std::vector<XferJob>& jobs);
  bool issue_some();
  void poll();
  bool idle() const;
  Layer& layer(LayerID id, int64_t size_hint = 0);
  bool ensure_chunk(Layer& L, LayerID id, int64_t c, bool want_landed);
  void stage_chunk(Layer& L, LayerID id, int64_t c);
  void landed(const Piece& p);
  hipEvent_t get_event();
  void put_event(hipEvent_t e);
  uint32_t crc_slot();
  void fail(const std::string& what);

  GpuEngineConfig cfg_;
  NodeID self_node_ = 0;
  std::map<NodeID, int> node_rank_;
  ncclComm_t comm_ = nullptr;
  hipStream_t comm_stream_ = nullptr, copy_stream_ = nullptr, verify_stream_ = nullptr;
  void* crc_ws_ = nullptr;
  uint32_t* crc_host_ = nullptr;  // pinned, mapped
  uint32_t* crc_dev_ = nullptr;   // device alias of crc_host_
  uint32_t crc_next_ = 0;
  static constexpr uint32_t kCrcSlots = 1u << 16;

  std::mutex req_mu_;
  std::condition_variable req_cv_, idle_cv_;
  std::deque<Req> reqs_;
  bool busy_ = false;  // issue thread has queued work or outstanding events

  // issue-thread state
  std::map<LayerID, Layer> layers_;
  std::deque<Piece> ops_;  // pending pieces in global key order
  std::deque<Verify> verifies_;
  std::deque<hipEvent_t> groups_inflight_;
  std::vector<hipEvent_t> event_pool_;
  std::map<uint64_t, int> batches_seen_;

  std::mutex stats_mu_;
  GpuEngineStats stats_;
  std::string error_;
  std::atomic<bool> failed_{false};
  std::thread th_;
};

// ---- raw device helpers for Python (pointers as integers)
std::shared_ptr<HostBuffer> alloc_pinned(int64_t size);
std::string nccl_unique_id();

}  // namespace dissem
