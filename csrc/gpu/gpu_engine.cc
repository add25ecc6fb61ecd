// RCCL-over-xGMI data engine (see gpu_engine.h for the execution model).
//
// Deadlock freedom. Every piece p has a global key k(p) = (batch, piece index
// within its job, job sequence number), known identically to its sender and
// receiver. Each rank posts its pieces in increasing key order, cut into
// consecutive ncclGroupStart/End groups on a single communicator/stream. A
// group finishes once every one of its pieces is posted by the partner rank.
// Suppose ranks were stuck: take the stuck group holding the smallest key k*
// among all unfinished pieces. Its partner has already posted every piece with
// a key < k* that it owns (they are finished, by minimality), so it reaches
// k* in its own order and posts it - contradiction. Hence no deadlock for any
// interleaving of batches the leader produces, including mode 2's dynamic
// dispatch. (Host-side waits never precede a post except for data that cannot
// exist yet, which the leader never schedules.)
#include "gpu/gpu_engine.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <set>

#include "core/crc32c.h"
#include "core/log.h"
#include "kernels/kernels.h"
#include "roles/node.h"

namespace dissem {

namespace {

#define HIP_OK(expr)                                                                                    \
  do {                                                                                                  \
    hipError_t _e = (expr);                                                                             \
    if (_e != hipSuccess) throw std::runtime_error(std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

#define NCCL_OK(expr)                                                                                      \
  do {                                                                                                     \
    ncclResult_t _r = (expr);                                                                              \
    if (_r != ncclSuccess) throw std::runtime_error(std::string(#expr " failed: ") + ncclGetErrorString(_r)); \
  } while (0)

}  // namespace

std::shared_ptr<HostBuffer> alloc_pinned(int64_t size) {
  void* p = nullptr;
  HIP_OK(hipHostMalloc(&p, size_t(std::max<int64_t>(size, 1)), hipHostMallocDefault));
  return HostBuffer::wrap(static_cast<uint8_t*>(p), size, std::shared_ptr<void>(p, [](void* q) { (void)hipHostFree(q); }));
}

std::string nccl_unique_id() {
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof id);
}

GpuEngine::GpuEngine(const GpuEngineConfig& cfg) : cfg_(cfg) {
  if (cfg_.world < 1 || cfg_.rank < 0 || cfg_.rank >= cfg_.world) throw std::runtime_error("bad rank/world");
  if (cfg_.rank_nodes.empty())
    for (int r = 0; r < cfg_.world; ++r) cfg_.rank_nodes.push_back(NodeID(r));
  if (int(cfg_.rank_nodes.size()) != cfg_.world) throw std::runtime_error("rank_nodes size != world");
  if (cfg_.chunk_bytes <= 0 || cfg_.chunk_bytes % 4096) throw std::runtime_error("chunk_bytes must be a multiple of 4 KiB");
  for (int r = 0; r < cfg_.world; ++r) node_rank_[cfg_.rank_nodes[size_t(r)]] = r;
  self_node_ = cfg_.rank_nodes[size_t(cfg_.rank)];
  HIP_OK(hipSetDevice(cfg_.device));
  HIP_OK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&verify_stream_, hipStreamNonBlocking));
  HIP_OK(hipMalloc(&crc_ws_, kern::crc32c_workspace_bytes(cfg_.chunk_bytes, cfg_.chunk_bytes)));
  HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&crc_host_), kCrcSlots * sizeof(uint32_t),
                       hipHostMallocMapped | hipHostMallocCoherent));
  HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&crc_dev_), crc_host_, 0));
  if (cfg_.world > 1) {
    if (cfg_.nccl_uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("nccl_uid must be ncclUniqueId bytes");
    ncclUniqueId id;
    memcpy(&id, cfg_.nccl_uid.data(), sizeof id);
    int64_t t0 = log::now_us();
    NCCL_OK(ncclCommInitRank(&comm_, cfg_.world, id, cfg_.rank));
    log::info(int64_t(self_node_)).i("world", cfg_.world).f("init_ms", double(log::now_us() - t0) / 1e3)
        .msg("rccl communicator ready");
  }
  th_ = std::thread([this] { run(); });
}

GpuEngine::~GpuEngine() { shutdown(); }

void GpuEngine::shutdown() {
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    if (!th_.joinable()) return;
    reqs_.push_back(Req{Req::Stop, {}, 0, 0, 0});
  }
  req_cv_.notify_all();
  th_.join();
  hipSetDevice(cfg_.device);
  hipStreamSynchronize(comm_stream_);
  hipStreamSynchronize(copy_stream_);
  hipStreamSynchronize(verify_stream_);
  if (comm_) {
    if (failed_) ncclCommAbort(comm_);
    else ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  for (auto& kv : layers_)
    if (kv.second.dev) hipFree(kv.second.dev);
  layers_.clear();
  for (auto e : event_pool_) hipEventDestroy(e);
  event_pool_.clear();
  if (crc_ws_) hipFree(crc_ws_);
  if (crc_host_) hipHostFree(crc_host_);
  crc_ws_ = nullptr;
  crc_host_ = nullptr;
  hipStreamDestroy(comm_stream_);
  hipStreamDestroy(copy_stream_);
  hipStreamDestroy(verify_stream_);
}

int GpuEngine::rank_of(NodeID n) const {
  auto it = node_rank_.find(n);
  if (it == node_rank_.end()) throw std::runtime_error("node " + std::to_string(n) + " has no rank");
  return it->second;
}

// --------------------------------------------------------------- setup API

GpuEngine::Layer& GpuEngine::layer(LayerID id, int64_t size_hint) {
  Layer& L = layers_[id];
  if (!L.size && size_hint) L.size = size_hint;
  int64_t n = L.size ? (L.size + cfg_.chunk_bytes - 1) / cfg_.chunk_bytes : 0;
  if (int64_t(L.st.size()) != n) {
    L.st.assign(size_t(n), L.seeded ? 2 : 0);
    L.ev.assign(size_t(n), nullptr);
    L.on_comm.assign(size_t(n), 0);
    L.want.assign(size_t(n), 0);
  }
  return L;
}

uint8_t* GpuEngine::provision(LayerID id, int64_t size) {
  std::lock_guard<std::mutex> lk(req_mu_);  // setup happens while the issue thread is idle
  Layer& L = layer(id, size);
  if (L.size != size) throw std::runtime_error("layer " + std::to_string(id) + " re-provisioned with another size");
  if (!L.dev) {
    HIP_OK(hipSetDevice(cfg_.device));
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, size_t(size)));
    L.dev = static_cast<uint8_t*>(p);
  }
  return L.dev;
}

uint8_t* GpuEngine::device_ptr(LayerID id) {
  std::lock_guard<std::mutex> lk(req_mu_);
  auto it = layers_.find(id);
  return it == layers_.end() ? nullptr : it->second.dev;
}

void GpuEngine::set_manifest(LayerID id, const CrcManifest& m) {
  std::lock_guard<std::mutex> lk(req_mu_);
  if (m.chunk_bytes != cfg_.chunk_bytes) throw std::runtime_error("manifest chunk_bytes must equal the engine chunk");
  layers_[id].manifest = m;
}

void GpuEngine::set_seeded(LayerID id, bool resident) {
  std::lock_guard<std::mutex> lk(req_mu_);
  Layer& L = layers_[id];
  L.seeded = resident;
  for (auto& s : L.st) s = resident ? 2 : 0;
}

std::map<LayerID, CrcManifest> GpuEngine::manifest() {
  std::lock_guard<std::mutex> lk(req_mu_);
  std::map<LayerID, CrcManifest> out;
  for (auto& kv : layers_)
    if (!kv.second.manifest.crc.empty()) out[kv.first] = kv.second.manifest;
  return out;
}

GpuEngineStats GpuEngine::stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return stats_;
}

std::string GpuEngine::error() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return error_;
}

void GpuEngine::fail(const std::string& what) {
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    if (error_.empty()) error_ = what;
  }
  failed_ = true;
  log::error(int64_t(self_node_)).s("error", what).msg("gpu engine failure");
  idle_cv_.notify_all();
}

// ------------------------------------------------------------ DataEngine

bool GpuEngine::on_message(const MessagePtr& m) {
  if (m->type != MsgType::XferBatch) return false;
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    Req r{Req::Batch, m->jobs, 0, 0, 0};
    reqs_.push_back(std::move(r));
  }
  req_cv_.notify_all();
  return true;
}

void GpuEngine::send_range(NodeID dest, LayerID layer_id, int64_t, int64_t, int64_t, int64_t) {
  log::error(int64_t(self_node_)).u("layer", layer_id).u("dest", dest)
      .msg("rccl engine is planned: sends are scheduled by the leader's XferBatch, not pushed");
}

void GpuEngine::load_range(LayerID layer_id, int64_t offset, int64_t size, int64_t total, int64_t) {
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    Req r{Req::Load, {}, layer_id, offset, size};
    (void)total;
    reqs_.push_back(std::move(r));
  }
  req_cv_.notify_all();
}

void GpuEngine::quiesce() {
  std::unique_lock<std::mutex> lk(req_mu_);
  idle_cv_.wait(lk, [&] { return (reqs_.empty() && !busy_) || failed_.load(); });
}

void GpuEngine::reset_session() {
  quiesce();
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    reqs_.push_back(Req{Req::Reset, {}, 0, 0, 0});
  }
  req_cv_.notify_all();
  quiesce();
  if (failed_) throw std::runtime_error("gpu engine failed: " + error());
}

// ------------------------------------------------------------ issue thread

hipEvent_t GpuEngine::get_event() {
  if (!event_pool_.empty()) {
    hipEvent_t e = event_pool_.back();
    event_pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}

void GpuEngine::put_event(hipEvent_t e) {
  if (e) event_pool_.push_back(e);
}

uint32_t GpuEngine::crc_slot() {
  uint32_t s = crc_next_;
  crc_next_ = (crc_next_ + 1) % kCrcSlots;
  return s;
}

bool GpuEngine::idle() const { return ops_.empty() && verifies_.empty() && groups_inflight_.empty(); }

void GpuEngine::landed(const Piece& p) {
  if (!node_) return;
  auto m = std::make_shared<Message>();
  m->type = MsgType::Landed;
  m->src = p.src_node;
  m->layer = p.layer;
  m->offset = p.off;
  m->data_size = p.len;
  m->total_size = p.total;
  node_->inject(m);
}

void GpuEngine::stage_chunk(Layer& L, LayerID id, int64_t c) {
  LayerSrc src;
  if (!node_ || !node_->store().get(id, &src) || !src.host)
    throw std::runtime_error("layer " + std::to_string(id) + " has no host source to stage");
  const int64_t off = c * cfg_.chunk_bytes;
  const int64_t len = std::min(cfg_.chunk_bytes, L.size - off);
  if (!L.dev) {
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, size_t(L.size)));  // unprovisioned slot (should not happen in benches)
    L.dev = static_cast<uint8_t*>(p);
  }
  HIP_OK(hipMemcpyAsync(L.dev + off, src.host->ptr + src.offset + off, size_t(len), hipMemcpyHostToDevice,
                        copy_stream_));
  hipEvent_t e = get_event();
  HIP_OK(hipEventRecord(e, copy_stream_));
  L.st[size_t(c)] = 1;
  L.ev[size_t(c)] = e;
  L.on_comm[size_t(c)] = 0;
  Verify v;
  Piece p{Kind::Local, 0, 0, cfg_.rank, id, off, len, L.size, c, true};
  p.src_node = self_node_;
  const bool check = cfg_.verify && int64_t(L.manifest.crc.size()) > c;
  if (check) {
    p.has_crc = true;
    p.crc = L.manifest.crc[size_t(c)];
    uint32_t slot = crc_slot();
    HIP_OK(hipStreamWaitEvent(verify_stream_, e, 0));
    HIP_OK(kern::crc32c_chunks(L.dev + off, len, len, crc_dev_ + slot, crc_ws_, verify_stream_));
    v.slots.push_back(slot);
    v.ev = get_event();
    HIP_OK(hipEventRecord(v.ev, verify_stream_));
  } else {
    v.slots.push_back(~0u);
    v.ev = get_event();
    HIP_OK(hipEventRecord(v.ev, copy_stream_));
  }
  v.pieces.push_back(p);
  verifies_.push_back(std::move(v));
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.bytes_staged += len;
}

bool GpuEngine::ensure_chunk(Layer& L, LayerID id, int64_t c, bool want_landed) {
  if (want_landed) L.want[size_t(c)] = 1;
  uint8_t s = L.st[size_t(c)];
  if (s == 2) {
    if (want_landed) {
      const int64_t off = c * cfg_.chunk_bytes;
      Piece p{Kind::Local, 0, 0, cfg_.rank, id, off, std::min(cfg_.chunk_bytes, L.size - off), L.size, c, true};
      p.src_node = self_node_;
      landed(p);
      L.want[size_t(c)] = 0;
    }
    return true;
  }
  if (s == 1) return true;
  LayerSrc src;
  if (node_ && node_->store().get(id, &src) && src.host) {
    stage_chunk(L, id, c);
    return true;
  }
  return false;
}

void GpuEngine::add_batch(std::vector<XferJob>& jobs) {
  std::sort(jobs.begin(), jobs.end(), [](const XferJob& a, const XferJob& b) { return a.seq < b.seq; });
  std::vector<Piece> pieces;
  const int64_t cb = cfg_.chunk_bytes;
  for (auto& j : jobs) {
    Kind kind;
    int peer;
    if (j.src == self_node_ && j.dst == self_node_) {
      kind = Kind::Local;
      peer = cfg_.rank;
    } else if (j.src == self_node_) {
      kind = Kind::Send;
      peer = rank_of(j.dst);
    } else if (j.dst == self_node_) {
      kind = Kind::Recv;
      peer = rank_of(j.src);
    } else {
      continue;
    }
    if (j.chunk_bytes && j.chunk_bytes != cb) {
      fail("job chunk grid " + std::to_string(j.chunk_bytes) + " != engine chunk " + std::to_string(cb));
      return;
    }
    Layer& L = layer(j.layer, j.total);
    if (L.size != j.total) {
      fail("layer " + std::to_string(j.layer) + " size mismatch");
      return;
    }
    const int64_t end = j.offset + j.size;
    const int64_t first_chunk = j.offset / cb;
    int64_t pidx = 0;
    for (int64_t pos = j.offset; pos < end; ++pidx) {
      const int64_t c = pos / cb;
      const int64_t cend = std::min((c + 1) * cb, L.size);
      const int64_t e = std::min(cend, end);
      Piece p{kind, j.seq, pidx, peer, j.layer, pos, e - pos, L.size, c, pos == c * cb && e == cend};
      p.src_node = j.src;
      const int64_t ci = c - first_chunk;
      if (p.full && ci < int64_t(j.crc.size())) {
        p.has_crc = true;
        p.crc = j.crc[size_t(ci)];
      }
      pieces.push_back(p);
      pos = e;
    }
  }
  std::stable_sort(pieces.begin(), pieces.end(), [](const Piece& a, const Piece& b) {
    return a.pidx != b.pidx ? a.pidx < b.pidx : a.seq < b.seq;
  });
  for (auto& p : pieces) {
    if (p.kind == Kind::Local) {
      // Local promotions do not take part in the RCCL order: stage right away so
      // PCIe runs ahead of the xGMI rounds that forward the same chunks.
      Layer& L = layer(p.layer);
      if (!ensure_chunk(L, p.layer, p.chunk, true)) fail("no source to load layer " + std::to_string(p.layer));
      continue;
    }
    ops_.push_back(p);
  }
}

bool GpuEngine::issue_some() {
  bool progress = false;
  const int per_peer = cfg_.group_peers > 0 ? cfg_.group_peers : 1;
  while (!ops_.empty() && int(groups_inflight_.size()) < cfg_.max_inflight_groups && !failed_) {
    std::vector<Piece> group;
    std::map<int, int> nsend, nrecv;
    std::set<std::pair<LayerID, int64_t>> recv_chunks;
    size_t take = 0;
    for (; take < ops_.size(); ++take) {
      Piece& p = ops_[take];
      if (p.kind == Kind::Send) {
        if (nsend[p.peer] >= per_peer) break;
        if (recv_chunks.count({p.layer, p.chunk})) break;  // forward only after the recv round is posted
        Layer& L = layer(p.layer);
        if (!ensure_chunk(L, p.layer, p.chunk, false)) break;  // data not here yet (and not stageable)
        nsend[p.peer]++;
      } else {
        if (nrecv[p.peer] >= per_peer) break;
        nrecv[p.peer]++;
        recv_chunks.insert({p.layer, p.chunk});
      }
      group.push_back(p);
    }
    if (group.empty()) break;
    ops_.erase(ops_.begin(), ops_.begin() + int64_t(take));
    int64_t t0 = log::now_us();
    // Cross-stream dependencies: sends of chunks still being staged on the copy stream.
    std::set<hipEvent_t> waits;
    for (auto& p : group) {
      if (p.kind != Kind::Send) continue;
      Layer& L = layers_[p.layer];
      if (L.st[size_t(p.chunk)] == 1 && !L.on_comm[size_t(p.chunk)] && L.ev[size_t(p.chunk)])
        waits.insert(L.ev[size_t(p.chunk)]);
    }
    for (auto e : waits) HIP_OK(hipStreamWaitEvent(comm_stream_, e, 0));
    int64_t sent = 0, recvd = 0;
    NCCL_OK(ncclGroupStart());
    for (auto& p : group) {
      Layer& L = layers_[p.layer];
      if (!L.dev) {
        void* q = nullptr;
        HIP_OK(hipMalloc(&q, size_t(L.size)));
        L.dev = static_cast<uint8_t*>(q);
      }
      if (p.kind == Kind::Send) {
        NCCL_OK(ncclSend(L.dev + p.off, size_t(p.len), ncclUint8, p.peer, comm_, comm_stream_));
        sent += p.len;
      } else {
        NCCL_OK(ncclRecv(L.dev + p.off, size_t(p.len), ncclUint8, p.peer, comm_, comm_stream_));
        recvd += p.len;
      }
    }
    NCCL_OK(ncclGroupEnd());
    hipEvent_t g = get_event();
    HIP_OK(hipEventRecord(g, comm_stream_));
    groups_inflight_.push_back(g);
    // Receivers: chunks become valid behind `g` on the comm stream; verify them.
    Verify v;
    bool any_recv = false;
    for (auto& p : group) {
      if (p.kind != Kind::Recv) continue;
      Layer& L = layers_[p.layer];
      L.st[size_t(p.chunk)] = 1;
      L.on_comm[size_t(p.chunk)] = 1;
      L.ev[size_t(p.chunk)] = nullptr;
      if (!any_recv) HIP_OK(hipStreamWaitEvent(verify_stream_, g, 0));
      any_recv = true;
      uint32_t slot = ~0u;
      if (cfg_.verify && p.has_crc && p.full) {
        slot = crc_slot();
        HIP_OK(kern::crc32c_chunks(L.dev + p.off, p.len, p.len, crc_dev_ + slot, crc_ws_, verify_stream_));
      }
      v.pieces.push_back(p);
      v.slots.push_back(slot);
    }
    if (any_recv) {
      v.ev = get_event();
      HIP_OK(hipEventRecord(v.ev, verify_stream_));
      verifies_.push_back(std::move(v));
    }
    {
      std::lock_guard<std::mutex> lk(stats_mu_);
      stats_.groups++;
      stats_.pieces += int64_t(group.size());
      stats_.bytes_sent += sent;
      stats_.bytes_recv += recvd;
      stats_.issue_ms += double(log::now_us() - t0) / 1e3;
    }
    progress = true;
  }
  return progress;
}

void GpuEngine::poll() {
  while (!groups_inflight_.empty()) {
    hipError_t r = hipEventQuery(groups_inflight_.front());
    if (r == hipErrorNotReady) break;
    if (r != hipSuccess) {
      fail(std::string("rccl group failed: ") + hipGetErrorString(r));
      return;
    }
    put_event(groups_inflight_.front());
    groups_inflight_.pop_front();
  }
  for (auto it = verifies_.begin(); it != verifies_.end();) {
    hipError_t r = hipEventQuery(it->ev);
    if (r == hipErrorNotReady) {
      ++it;
      continue;
    }
    if (r != hipSuccess) {
      fail(std::string("landing failed: ") + hipGetErrorString(r));
      return;
    }
    for (size_t i = 0; i < it->pieces.size(); ++i) {
      const Piece& p = it->pieces[i];
      Layer& L = layers_[p.layer];
      if (it->slots[i] != ~0u) {
        uint32_t got = __atomic_load_n(&crc_host_[it->slots[i]], __ATOMIC_ACQUIRE);
        if (got != p.crc) {
          {
            std::lock_guard<std::mutex> lk(stats_mu_);
            stats_.verify_failures++;
          }
          char buf[160];
          snprintf(buf, sizeof buf, "CRC32C mismatch layer %llu chunk %lld: got %08x want %08x",
                   (unsigned long long)p.layer, (long long)p.chunk, got, p.crc);
          fail(buf);
          return;
        }
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.bytes_verified += p.len;
      } else if (p.kind == Kind::Recv) {
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.unverified_pieces++;
      }
      if (p.full) L.st[size_t(p.chunk)] = 2;
      if (L.ev[size_t(p.chunk)]) {
        put_event(L.ev[size_t(p.chunk)]);
        L.ev[size_t(p.chunk)] = nullptr;
      }
      if (p.kind == Kind::Recv) {
        landed(p);
      } else if (L.want[size_t(p.chunk)]) {
        landed(p);
        L.want[size_t(p.chunk)] = 0;
      }
    }
    put_event(it->ev);
    it = verifies_.erase(it);
  }
}

void GpuEngine::take_requests(bool block) {
  std::deque<Req> got;
  {
    std::unique_lock<std::mutex> lk(req_mu_);
    if (block && reqs_.empty()) {
      busy_ = false;
      idle_cv_.notify_all();
      req_cv_.wait_for(lk, std::chrono::milliseconds(50), [&] { return !reqs_.empty(); });
    }
    got.swap(reqs_);
    if (!got.empty()) busy_ = true;
  }
  for (auto& r : got) {
    switch (r.type) {
      case Req::Batch:
        add_batch(r.jobs);
        break;
      case Req::Load: {
        Layer& L = layer(r.layer);
        if (!L.size) break;
        for (int64_t c = r.off / cfg_.chunk_bytes; c * cfg_.chunk_bytes < r.off + r.len && c < int64_t(L.st.size()); ++c)
          if (!ensure_chunk(L, r.layer, c, true)) fail("no source to load layer " + std::to_string(r.layer));
        break;
      }
      case Req::Reset: {
        for (auto& kv : layers_) {
          Layer& L = kv.second;
          for (size_t c = 0; c < L.st.size(); ++c) {
            L.st[c] = L.seeded ? 2 : 0;
            if (L.ev[c]) put_event(L.ev[c]);
            L.ev[c] = nullptr;
            L.on_comm[c] = 0;
            L.want[c] = 0;
          }
          if (cfg_.poison && !L.seeded && L.dev) HIP_OK(hipMemsetAsync(L.dev, 0, size_t(L.size), comm_stream_));
        }
        HIP_OK(hipStreamSynchronize(comm_stream_));
        break;
      }
      case Req::Quiesce:
        break;
      case Req::Stop: {
        std::lock_guard<std::mutex> lk(req_mu_);
        reqs_.push_front(r);  // seen by run()
        return;
      }
    }
  }
}

void GpuEngine::run() {
  try {
    HIP_OK(hipSetDevice(cfg_.device));
    int64_t last_async_check = log::now_us();
    for (;;) {
      const bool work = !idle();
      take_requests(!work);
      {
        std::lock_guard<std::mutex> lk(req_mu_);
        if (!reqs_.empty() && reqs_.front().type == Req::Stop) break;
      }
      if (failed_) {
        // Drop queued work; keep serving Stop. (In-flight RCCL ops are aborted at shutdown.)
        ops_.clear();
        verifies_.clear();
        groups_inflight_.clear();
        std::lock_guard<std::mutex> lk(req_mu_);
        busy_ = false;
        idle_cv_.notify_all();
        continue;
      }
      bool progress = issue_some();
      poll();
      {
        std::lock_guard<std::mutex> lk(req_mu_);
        busy_ = !idle() || !reqs_.empty();
        if (!busy_) idle_cv_.notify_all();
      }
      if (comm_ && log::now_us() - last_async_check > 100000) {
        last_async_check = log::now_us();
        ncclResult_t ar = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress)
          fail(std::string("rccl async error: ") + ncclGetErrorString(ar));
      }
      if (!progress && !idle()) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  } catch (const std::exception& e) {
    fail(e.what());
    std::lock_guard<std::mutex> lk(req_mu_);
    busy_ = false;
    idle_cv_.notify_all();
  }
}

}  // namespace dissem
