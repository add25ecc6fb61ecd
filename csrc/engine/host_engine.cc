// Host data engine: layer payloads in host memory or files, pushed as Layer
// messages over the node's transport (reference: transport.go:308-373 for the
// send side, node.go:1592-1643 for ranges; the mode-3 "client simulation"
// rate-limited copy is node.go:1609-1634).
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>

#include "core/log.h"
#include "core/ratelimit.h"
#include "engine/engine.h"
#include "roles/node.h"

namespace dissem {

void WorkerSet::spawn(std::function<void()> fn) {
  active_++;
  std::thread([this, fn = std::move(fn)] {
    try {
      fn();
    } catch (const std::exception& e) {
      log::error(-1).s("error", e.what()).msg("worker failed");
    }
    std::lock_guard<std::mutex> lk(mu_);
    active_--;
    cv_.notify_all();
  }).detach();
}

void WorkerSet::join_all() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return active_.load() == 0; });
}

namespace {

class HostEngine : public DataEngine {
 public:
  explicit HostEngine(std::map<NodeID, int64_t> link_rate) : link_rate_(std::move(link_rate)) {}
  ~HostEngine() override { workers_.join_all(); }
  std::string name() const override { return "host"; }
  Location target() const override { return Location::Inmem; }

  void send_range(NodeID dest, LayerID layer, int64_t offset, int64_t size, int64_t total, int64_t rate) override {
    LayerSrc src;
    if (!node_->store().get(layer, &src)) return;
    Node* node = node_;
    if (auto it = link_rate_.find(dest); it != link_rate_.end() && it->second > 0)
      rate = rate > 0 ? std::min(rate, it->second) : it->second;
    workers_.spawn([node, dest, layer, offset, size, total, rate, src] {
      Message lm;
      lm.type = MsgType::Layer;
      lm.src = node->id();
      lm.epoch = node->epoch();
      lm.layer = layer;
      lm.data_size = size;
      lm.total_size = total;
      lm.offset = offset;
      lm.rate = rate;
      LayerPayload p;
      if (src.host) {
        p.host = src.host;
        p.host_off = src.offset + offset;
      } else if (!src.path.empty()) {
        p.path = src.path;
        p.file_off = src.offset + offset;
      } else {
        log::error(int64_t(node->id())).msg("unknown error sending layer " + std::to_string(layer));
        return;
      }
      int64_t t0 = log::now_us();
      try {
        node->transport()->send(dest, lm, &p);
      } catch (const std::exception& e) {
        log::error(int64_t(node->id())).s("error", e.what()).msg("couldn't send a layer " + std::to_string(layer));
        return;
      }
      double secs = double(log::now_us() - t0) / 1e6;
      log::info(int64_t(node->id())).u("layer", layer).u("dest", dest).f("send_dur[s]", secs)
          .f("throughput[MiB/s]", secs > 0 ? double(size) / secs / 1048576.0 : 0.0)  // quirk Q11 guarded
          .msg("finished sending layer");
    });
  }

  void load_range(LayerID layer, int64_t offset, int64_t size, int64_t total, int64_t rate) override {
    // Promote a disk (or other host) copy into host memory, paced at `rate`.
    LayerSrc src;
    if (!node_->store().get(layer, &src)) return;
    Node* node = node_;
    workers_.spawn([node, layer, offset, size, total, rate, src] {
      int64_t t0 = log::now_us();
      uint8_t* dst = node->store().host_landing(layer, total);
      TokenBucket tb(rate);
      if (src.host && src.host->ptr != dst) {
        tb.paced(size, [&](int64_t off, int64_t n) {
          memcpy(dst + offset + off, src.host->ptr + src.offset + offset + off, size_t(n));
        });
      } else if (!src.host && !src.path.empty()) {
        int fd = ::open(src.path.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) throw std::runtime_error("open " + src.path);
        tb.paced(size, [&](int64_t off, int64_t n) {
          int64_t done = 0;
          while (done < n) {
            ssize_t r = ::pread(fd, dst + offset + off + done, size_t(n - done), off_t(src.offset + offset + off + done));
            if (r <= 0) {
              ::close(fd);
              throw std::runtime_error("short read " + src.path);
            }
            done += r;
          }
        });
        ::close(fd);
      } else if (src.host && src.host->ptr == dst) {
        tb.paced(size, [](int64_t, int64_t) {});  // already in place; only the pacing is simulated
      }
      auto m = std::make_shared<Message>();
      m->type = MsgType::Landed;
      m->src = node->id();
      m->layer = layer;
      m->offset = offset;
      m->data_size = size;
      m->total_size = total;
      m->dur_ms = double(log::now_us() - t0) / 1e3;
      node->inject(m);
    });
  }

  void quiesce() override { workers_.join_all(); }
  void shutdown() override { workers_.join_all(); }

 private:
  std::map<NodeID, int64_t> link_rate_;
  WorkerSet workers_;
};

}  // namespace

std::shared_ptr<DataEngine> make_host_engine(const std::map<NodeID, int64_t>& link_rate) {
  return std::make_shared<HostEngine>(link_rate);
}

}  // namespace dissem
