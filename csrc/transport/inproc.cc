// In-process transport: the test fake (reference: transport.go:493-631).
//
// Nodes in one process exchange MessagePtrs through a process-global registry
// keyed by address. Layer payloads are passed by pointer (no serialization),
// like the reference; the receiving node copies them into its store. Pipes
// forward a client-provided layer onward, mirroring the TCP tee.
#include <atomic>
#include <memory>

#include "core/log.h"
#include "transport/transport.h"

namespace dissem {

namespace {

class InprocTransport;
std::mutex g_reg_mu;
std::map<std::string, std::weak_ptr<InprocTransport>> g_registry;

class InprocTransport : public Transport, public std::enable_shared_from_this<InprocTransport> {
 public:
  explicit InprocTransport(std::string addr) : addr_(std::move(addr)) {}

  void send(NodeID dest, const Message& m, const LayerPayload* payload) override {
    std::string daddr;
    if (!lookup(dest, &daddr)) daddr = std::to_string(dest);  // transport.go:545-547
    std::shared_ptr<InprocTransport> peer;
    {
      std::lock_guard<std::mutex> lk(g_reg_mu);
      auto it = g_registry.find(daddr);
      if (it != g_registry.end()) peer = it->second.lock();
    }
    if (!peer) throw std::runtime_error("peer " + daddr + " not found");
    auto msg = std::make_shared<Message>(m);
    if (m.type == MsgType::Layer) {
      // Materialize the payload as a host buffer reference (no byte copy when in memory).
      if (payload && payload->host) {
        msg->data = payload->host;
        msg->data_off = payload->host_off;
      } else if (payload && !payload->path.empty()) {
        auto buf = HostBuffer::alloc(m.data_size, false);
        FILE* f = fopen(payload->path.c_str(), "rb");
        if (!f) throw std::runtime_error("open " + payload->path);
        fseek(f, long(payload->file_off), SEEK_SET);
        size_t got = fread(buf->ptr, 1, size_t(m.data_size), f);
        fclose(f);
        if (int64_t(got) != m.data_size) throw std::runtime_error("short read " + payload->path);
        msg->data = buf;
        msg->data_off = 0;
      }
      bytes_sent += m.data_size;
      peer->bytes_received += m.data_size;
      peer->maybe_pipe(*msg);
    }
    peer->inbox_.push(msg);
  }

  void broadcast(const Message& m) override {
    std::vector<std::pair<std::string, std::shared_ptr<InprocTransport>>> peers;
    {
      std::lock_guard<std::mutex> lk(g_reg_mu);
      for (auto& kv : g_registry)
        if (auto p = kv.second.lock()) peers.emplace_back(kv.first, p);
    }
    for (auto& pr : peers) {
      if (pr.first == addr_) continue;  // transport.go:583-585
      pr.second->inbox_.push(std::make_shared<Message>(m));
    }
  }

  void register_pipe(LayerID layer, NodeID dest) override {
    std::lock_guard<std::mutex> lk(pipe_mu_);
    if (pipes_.count(layer)) throw std::runtime_error("pipe already registered");
    pipes_[layer] = dest;
  }

  std::string address() const override { return addr_; }

  bool alive(NodeID id) override {
    std::string daddr;
    if (!lookup(id, &daddr)) daddr = std::to_string(id);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_registry.find(daddr);
    return it != g_registry.end() && it->second.lock() != nullptr;
  }

  void close() override {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_registry.find(addr_);
    if (it != g_registry.end() && it->second.lock().get() == this) g_registry.erase(it);
    inbox_.close();
  }

 private:
  // Forward a layer received from the client to the registered pipe dest.
  void maybe_pipe(const Message& m) {
    NodeID dest;
    {
      std::lock_guard<std::mutex> lk(pipe_mu_);
      auto it = pipes_.find(m.layer);
      if (it == pipes_.end()) return;
      dest = it->second;
      pipes_.erase(it);
    }
    LayerPayload p;
    p.host = m.data;
    p.host_off = m.data_off;
    send(dest, m, &p);
  }

  std::string addr_;
  std::mutex pipe_mu_;
  std::map<LayerID, NodeID> pipes_;
};

}  // namespace

std::shared_ptr<Transport> make_inproc_transport(const std::string& addr, const AddrRegistry& reg) {
  auto t = std::make_shared<InprocTransport>(addr);
  t->set_registry(reg);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  g_registry[addr] = t;
  return t;
}

}  // namespace dissem
