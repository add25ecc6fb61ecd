// Data engines: how layer bytes move once the control plane has decided who
// sends what (reference: the layer branch of TcpTransport.Send,
// transport.go:258-373, and handleFlowRetransmit, node.go:1592-1643).
//
//  * HostEngine  - bytes in host memory / files, pushed as Layer messages over
//                  the node's Transport (TCP: fresh connection per payload,
//                  in-proc: pointer hand-off). Target tier: host RAM.
//  * PlannedEngine (planned_engine.h) - bytes in HBM, moved by leader-planned
//                  grouped RCCL point-to-point rounds over xGMI (HipBackend) or a
//                  simulated fabric (SimBackend); staging from host/NVMe on a copy
//                  queue; CRC32C verification by a gfx950 kernel. Target: Device.
//
// Engines report completions by injecting MsgType::Landed into the owning
// node's inbox, so every role state transition happens on the node's single
// event-loop thread.
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <thread>

#include "core/types.h"
#include "core/wire.h"

namespace dissem {

class Node;

class DataEngine {
 public:
  virtual ~DataEngine() = default;
  virtual void bind(Node* node) { node_ = node; }
  // Push [offset, offset+size) of `layer` (total bytes `total`) to `dest`, paced at `rate` (0 = unlimited).
  virtual void send_range(NodeID dest, LayerID layer, int64_t offset, int64_t size, int64_t total,
                          int64_t rate) = 0;
  // Make [offset, offset+size) of `layer` resident in this node's target tier.
  virtual void load_range(LayerID layer, int64_t offset, int64_t size, int64_t total, int64_t rate) = 0;
  // Host bytes of `layer` (a client stream landing in place at `base`) are
  // present up to `prefix` of its `total` source bytes: cut-through engines
  // may stage those chunks now.
  virtual void host_prefix_ready(LayerID layer, const uint8_t* base, int64_t prefix, int64_t total) {
    (void)layer;
    (void)base;
    (void)prefix;
    (void)total;
  }
  // Engine-specific control messages (GPU layer headers). Return true if consumed.
  virtual bool on_message(const MessagePtr&) { return false; }
  // Collective broadcast of a whole layer from this node to `dests` (GPU mode 0).
  virtual bool supports_broadcast() const { return false; }
  virtual void broadcast_layer(LayerID, int64_t, const std::vector<NodeID>&) {}
  // Planned engines (GPU) do not take per-message pushes: the leader batches
  // sequence-numbered XferJobs and sends each rank its share (MsgType::XferBatch).
  virtual bool planned() const { return false; }
  virtual int64_t chunk_bytes() const { return 0; }
  // Per-layer CRC manifests of layers this rank can serve (sent with Announce).
  virtual std::map<LayerID, CrcManifest> manifest() { return {}; }
  // Elastic recovery (leader): a fresh communicator id the survivors re-form
  // around (RCCL: ncclGetUniqueId bytes); "" when the engine needs none.
  virtual std::string new_comm_id() { return ""; }
  // Wait until every transfer this engine started for its node has finished.
  virtual void quiesce() {}
  virtual void shutdown() {}
  virtual std::string name() const = 0;
  virtual Location target() const = 0;

 protected:
  Node* node_ = nullptr;
};

// Tracks detached worker threads (the reference's per-send goroutines) so
// shutdown can wait for them.
class WorkerSet {
 public:
  ~WorkerSet() { join_all(); }
  void spawn(std::function<void()> fn);
  void join_all();
  int active() const { return active_.load(); }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<int> active_{0};
};

// `link_rate`: per-destination pacing cap in B/s (fault injection
// --inject slow-link=S,D,RATE on sender S); 0 / absent = unlimited.
std::shared_ptr<DataEngine> make_host_engine(const std::map<NodeID, int64_t>& link_rate = {});

}  // namespace dissem
