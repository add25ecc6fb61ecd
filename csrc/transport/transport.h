// Control-plane transport (reference: distributor/transport.go:18-25).
//
// A Transport delivers decoded Messages into an inbox queue. Two
// implementations: TcpTransport (JSON envelopes on persistent connections, a
// fresh connection per layer payload, token-bucket pacing, cut-through "pipe")
// and InprocTransport (a process-global registry of queues; the test fake).
// On MI355X the layer bytes normally move on the RCCL data plane instead
// (csrc/engine/planned_engine.cc on csrc/gpu/hip_backend.cc); the TCP payload path is the CPU/loopback plane.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "core/queue.h"
#include "core/wire.h"

namespace dissem {

using AddrRegistry = std::map<NodeID, std::string>;  // transport.go:57

// Layer-send source descriptor: bytes from host memory or a file range.
struct LayerPayload {
  std::shared_ptr<HostBuffer> host;  // if set: bytes at host->ptr + host_off
  int64_t host_off = 0;
  std::string path;                  // else: file, read at file_off
  int64_t file_off = 0;
};

// Receiver-side landing: given a Layer header, return where its bytes go
// (host memory, at least data_size bytes), or nullptr to allocate a buffer.
using LandingFn = std::function<uint8_t*(const Message& hdr)>;
// Receiver-side progress of an in-place landing: `got` bytes of the range have
// arrived (called from the reader thread as they come in; cut-through).
using ProgressFn = std::function<void(const Message& hdr, int64_t got)>;

class Transport {
 public:
  virtual ~Transport() = default;
  // Control message or (for MsgType::Layer) header + payload.
  virtual void send(NodeID dest, const Message& m, const LayerPayload* payload = nullptr) = 0;
  // Several control messages at once (the leader's per-rank transfer batches):
  // TCP encodes them all before the first write, so no peer starts working
  // (and competing for the CPU) while the rest are still being encoded.
  // Throws on the first failed send, after trying the others.
  virtual void send_many(std::vector<std::pair<NodeID, Message>>& msgs) {
    std::string err;
    for (auto& m : msgs) {
      try {
        send(m.first, m.second);
      } catch (const std::exception& e) {
        if (err.empty()) err = e.what();
      }
    }
    if (!err.empty()) throw std::runtime_error(err);
  }
  virtual void register_pipe(LayerID layer, NodeID dest) = 0;
  virtual void broadcast(const Message& m) = 0;
  virtual std::string address() const = 0;
  virtual void close() = 0;
  // Liveness probe used by the leader's failure detector: can `id` still be
  // reached (TCP: a fresh connect succeeds; in-process: its endpoint exists)?
  virtual bool alive(NodeID id) { return true; }
  // Open the cached control connection to `id` ahead of the first message (the
  // leader does this when a peer announces, so the first dispatch after "timer
  // start" pays no connect). Best effort: errors surface on the first send.
  virtual void warm(NodeID id) {}

  BlockingQueue<MessagePtr>& deliver() { return inbox_; }
  // Node-internal events (engine completions) enter the same inbox.
  void inject(MessagePtr m) { inbox_.push(std::move(m)); }

  void set_registry(const AddrRegistry& reg) {
    std::lock_guard<std::mutex> lk(reg_mu_);
    registry_ = reg;
  }
  void add_peer(NodeID id, const std::string& addr) {
    std::lock_guard<std::mutex> lk(reg_mu_);
    registry_[id] = addr;
  }
  AddrRegistry registry() const {
    std::lock_guard<std::mutex> lk(reg_mu_);
    return registry_;
  }
  // Receiver hooks of the node that currently runs on this transport (one
  // node per session, the transport outlives it): `owner` tags them so a
  // finished node clears only its own.
  void set_hooks(const void* owner, LandingFn landing, ProgressFn progress) {
    std::lock_guard<std::mutex> lk(reg_mu_);
    hook_owner_ = owner;
    landing_ = std::move(landing);
    progress_ = std::move(progress);
  }
  void clear_hooks(const void* owner) {
    std::lock_guard<std::mutex> lk(reg_mu_);
    if (hook_owner_ != owner) return;
    hook_owner_ = nullptr;
    landing_ = nullptr;
    progress_ = nullptr;
  }

  // Counters for observability.
  std::atomic<int64_t> bytes_sent{0};
  std::atomic<int64_t> bytes_received{0};

  // Limits on what a peer may make this transport buffer (TCP): one control
  // envelope, and one layer message's payload (its DataSize / TotalSize - the
  // runtime sets the largest layer of its config). A peer past either is
  // disconnected before anything is allocated.
  static constexpr int64_t kDefaultMaxEnvelope = 64ll << 20;
  static constexpr int64_t kDefaultMaxPayload = 64ll << 30;
  void set_max_envelope(int64_t n) { max_envelope_ = n; }
  void set_max_payload(int64_t n) { max_payload_ = n; }

 protected:
  bool lookup(NodeID id, std::string* addr) const {
    std::lock_guard<std::mutex> lk(reg_mu_);
    auto it = registry_.find(id);
    if (it == registry_.end()) return false;
    *addr = it->second;
    return true;
  }
  LandingFn landing() const {
    std::lock_guard<std::mutex> lk(reg_mu_);
    return landing_;
  }
  ProgressFn progress() const {
    std::lock_guard<std::mutex> lk(reg_mu_);
    return progress_;
  }

  mutable std::mutex reg_mu_;
  AddrRegistry registry_;
  const void* hook_owner_ = nullptr;
  LandingFn landing_;
  ProgressFn progress_;
  BlockingQueue<MessagePtr> inbox_;
  std::atomic<int64_t> max_envelope_{kDefaultMaxEnvelope};
  std::atomic<int64_t> max_payload_{kDefaultMaxPayload};
};

std::shared_ptr<Transport> make_inproc_transport(const std::string& addr, const AddrRegistry& reg);
std::shared_ptr<Transport> make_tcp_transport(const std::string& addr, const AddrRegistry& reg,
                                              bool is_client = false);

}  // namespace dissem
