// Planned data engine (see planned_engine.h).
//
// Deadlock freedom. Every piece p has a global key k(p) = (batch, chunk index
// within its layer, job sequence number), known identically to its sender and
// receiver, and a lane (lane_of the directed pair, also identical on both
// ends). Each rank posts the pieces of each lane in increasing key order, cut
// into consecutive groups on that lane's ordered queue; a P2P op inside a group
// progresses as soon as its partner's op is posted. Suppose ranks were stuck:
// take the unfinished piece with the smallest key k*, on lane x. On both of its
// ranks every earlier group of lane x holds only keys < k* (consecutive
// segments of the key order), which finished by minimality, so both ranks
// reach and post the group holding k* - unless a host- or device-side wait
// holds it back. Waits point only at smaller keys: a send waits for staging
// (no comm dependency) or, when it forwards a chunk this rank receives on
// another lane, for a mark recorded after that recv's group; a group that
// receives a chunk with a queued forward is closed right after that recv, so
// the mark covers keys <= the recv's key < the forward's key. When both ends
// hold a layer, a rank can be asked to send a chunk (key k1) and to receive
// it (key k2 > k1) in one batch on two lanes; the recv is then not posted
// before that send, which stages from the local copy, so the send never
// waits on the recv (the recv's host-side wait is on the posting of a
// smaller key, which needs only smaller keys). Those finished
// too, so k* completes - a contradiction. Hence no deadlock for any
// interleaving of batches (mode 2's dynamic dispatch included) and any number
// of lanes. tests/test_planned_sim.py checks this on the simulated fabric for
// every mode at up to 8 ranks, with one lane and with world-1 lanes.
#include "engine/planned_engine.h"

#include <execinfo.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <set>

#include "core/fp8.h"
#include "core/log.h"
#include "core/queue.h"
#include "core/trace.h"
#include "roles/node.h"

namespace dissem {

namespace {
// Diagnostics: the monitor asks a stuck issue thread for its native stack
// (async-signal-safe: backtrace + backtrace_symbols_fd straight to stderr;
// resolve the .so offsets with addr2line).
void dump_stack_handler(int) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  static const char hdr[] = "=== issue thread stack ===\n";
  (void)!write(2, hdr, sizeof hdr - 1);
  backtrace_symbols_fd(frames, n, 2);
}

size_t log2_bucket(double since) {
  const int64_t us = int64_t((vclock::now() - since) * 1e6);
  size_t b = 0;
  while (b < 31 && (int64_t(1) << (b + 1)) <= us) ++b;
  return b;
}
}  // namespace

PlannedEngine::PlannedEngine(const PlannedConfig& cfg, std::unique_ptr<Backend> backend)
    : cfg_(cfg), backend_(std::move(backend)) {
  if (cfg_.world < 1 || cfg_.rank < 0 || cfg_.rank >= cfg_.world) throw std::runtime_error("bad rank/world");
  if (cfg_.rank_nodes.empty())
    for (int r = 0; r < cfg_.world; ++r) cfg_.rank_nodes.push_back(NodeID(r));
  if (int(cfg_.rank_nodes.size()) != cfg_.world) throw std::runtime_error("rank_nodes size != world");
  if (cfg_.chunk_bytes <= 0 || cfg_.chunk_bytes % 4096)
    throw std::runtime_error("chunk_bytes must be a positive multiple of 4 KiB");
  if (cfg_.group_peers < 1) cfg_.group_peers = 1;
  grid_ = cfg_.chunk_bytes;
  if (cfg_.pack == 1) {
    fp8::check(cfg_.chunk_bytes, cfg_.chunk_bytes, cfg_.pack_block);
    grid_ = fp8::packed_chunk(cfg_.chunk_bytes, cfg_.pack_block);
  } else if (cfg_.pack != 0) {
    throw std::runtime_error("unknown pack format " + std::to_string(cfg_.pack));
  }
  if (cfg_.unpack_store && cfg_.pack != 1) throw std::runtime_error("unpack_store needs pack = fp8");
  inject_rng_.seed(cfg_.inject_seed * 0x9E3779B97F4A7C15ull + uint64_t(cfg_.rank));
  lanes_ = std::max(1, backend_->lanes());
  ops_.resize(size_t(lanes_));
  inflight_.resize(size_t(lanes_));
  stats_.lanes = lanes_;
  stats_.lane_busy_ms.assign(size_t(lanes_), 0.0);
  stats_.comm_init_ms = backend_->comm_init_ms();
  stats_.comm_connect_ms = backend_->comm_connect_ms();
  stats_.lane_init_ms = backend_->lane_init_ms();
  stats_.lane_connect_ms = backend_->lane_connect_ms();
  for (int r = 0; r < cfg_.world; ++r) node_rank_[cfg_.rank_nodes[size_t(r)]] = r;
  self_node_ = cfg_.rank_nodes[size_t(cfg_.rank)];
  th_ = vclock::spawn([this] { run(); }, "engine-issue");
  monitor_ = vclock::spawn([this] { monitor_loop(); }, "engine-monitor");
}

void PlannedEngine::monitor_loop() {
  int64_t reported = 0;
  while (!stop_req_) {
    vclock::sleep_for(0.25);
    {
      // the issue thread loops every ~20 us while it has work: a loop counter that
      // stands still for 5 s means it is stuck outside any marked backend call
      const int64_t t = loop_ticks_.load();
      const double now = vclock::now();
      if (t != last_ticks_) {
        last_ticks_ = t;
        ticks_since_ = now;
      } else if (now - ticks_since_ > 5.0 && !call_what_.load() && !idle_flag_.load()) {
        ticks_since_ = now;
        log::warn(int64_t(self_node_)).i("loop_ticks", t).msg("issue thread not looping (stuck outside backend calls)");
        if (!stack_dumped_ && getenv("DISSEM_STACK_DUMP")) {
          stack_dumped_ = true;
          struct sigaction sa {};
          sa.sa_handler = dump_stack_handler;
          sigemptyset(&sa.sa_mask);
          sigaction(SIGUSR2, &sa, nullptr);
          pthread_kill(th_.native_handle(), SIGUSR2);
        }
      }
    }
    const char* what = call_what_.load();
    const int64_t since = call_since_us_.load();
    if (!what || since == reported) continue;
    const double age = double(CallMark::now_us() - since) / 1e6;
    if (age < 3.0) continue;
    reported = since;
    log::warn(int64_t(self_node_)).s("call", what).i("lane", call_lane_.load()).f("seconds", age)
        .msg("issue thread blocked inside a backend call");
  }
}

PlannedEngine::~PlannedEngine() { shutdown(); }

void PlannedEngine::shutdown() {
  if (stopped_.exchange(true)) return;
  stop_req_ = true;
  req_cv_.notify_all();
  if (th_.joinable()) th_.join();
  if (monitor_.joinable()) monitor_.join();
  disk_cv_.notify_all();
  for (auto& t : readers_) t.join();
  readers_.clear();
  idle_cv_.notify_all();
  backend_->sync_all();
  if (pacer_) {
    pacer_.reset();
    NodePacer::unlink(cfg_.node_disk_key.empty() ? "default" : cfg_.node_disk_key);
  }
  for (auto* b : bounce_all_) backend_->free_host(b);
  bounce_all_.clear();
  bounce_free_.clear();
  for (auto& kv : layers_) {
    if (kv.second.dev) backend_->free(kv.second.dev);
    if (kv.second.out) backend_->free(kv.second.out);
  }
  layers_.clear();
  for (uint8_t* b : scratch_all_) backend_->free(b);
  scratch_all_.clear();
  scratch_free_.clear();
  backend_->destroy(failed_.load());
}

uint8_t* PlannedEngine::scratch_take() {
  if (!scratch_free_.empty()) {
    uint8_t* b = scratch_free_.back();
    scratch_free_.pop_back();
    return b;
  }
  CallMark cm(this, "alloc", -1);
  scratch_all_.push_back(backend_->alloc(cfg_.chunk_bytes));  // a full piece is at most one chunk
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.scratch_buffers++;
  }
  return scratch_all_.back();
}

int PlannedEngine::rank_of(NodeID n) const {
  auto it = node_rank_.find(n);
  if (it == node_rank_.end()) throw std::runtime_error("node " + std::to_string(n) + " has no rank");
  return it->second;
}

// --------------------------------------------------------------- setup API

int64_t PlannedEngine::slot_size(int64_t src_bytes) const {
  if (cfg_.pack == 1) {
    fp8::check(src_bytes, cfg_.chunk_bytes, cfg_.pack_block);
    return fp8::packed_size(src_bytes, cfg_.chunk_bytes, cfg_.pack_block);
  }
  return src_bytes;
}

int64_t PlannedEngine::src_len(const Layer& L, int64_t c) const {
  if (cfg_.pack == 1 && !L.src_packed) {
    const int64_t src = fp8::source_size(L.size, cfg_.chunk_bytes, cfg_.pack_block);
    return std::min(cfg_.chunk_bytes, src - c * cfg_.chunk_bytes);
  }
  return std::min(grid_, L.size - c * grid_);
}

PlannedEngine::Layer& PlannedEngine::layer(LayerID id, int64_t size_hint) {
  Layer& L = layers_[id];
  if (!L.size && size_hint) L.size = size_hint;
  int64_t n = L.size ? (L.size + grid_ - 1) / grid_ : 0;
  if (int64_t(L.st.size()) != n) {
    L.st.assign(size_t(n), L.seeded ? 2 : 0);
    L.ev.assign(size_t(n), 0);
    L.rkey.assign(size_t(n), Key{});
    L.want.assign(size_t(n), 0);
    L.fails.assign(size_t(n), 0);
  }
  return L;
}

uint8_t* PlannedEngine::provision(LayerID id, int64_t size) {
  std::lock_guard<std::mutex> lk(req_mu_);  // setup runs while the issue thread is idle
  if (cfg_.pack == 1) (void)fp8::source_size(size, cfg_.chunk_bytes, cfg_.pack_block);  // must be a packed size
  Layer& L = layer(id, size);
  if (L.size != size) throw std::runtime_error("layer " + std::to_string(id) + " re-provisioned with another size");
  if (!L.dev) L.dev = backend_->alloc(size);
  return L.dev;
}

uint8_t* PlannedEngine::unpacked_ptr(LayerID id) {
  std::lock_guard<std::mutex> lk(req_mu_);
  auto it = layers_.find(id);
  return it == layers_.end() ? nullptr : it->second.out;
}

uint8_t* PlannedEngine::device_ptr(LayerID id) {
  std::lock_guard<std::mutex> lk(req_mu_);
  auto it = layers_.find(id);
  return it == layers_.end() ? nullptr : it->second.dev;
}

void PlannedEngine::set_manifest(LayerID id, const CrcManifest& m) {
  std::lock_guard<std::mutex> lk(req_mu_);
  if (m.chunk_bytes != grid_) throw std::runtime_error("manifest chunk_bytes must equal the engine chunk grid");
  layers_[id].manifest = m;
}

void PlannedEngine::set_seeded(LayerID id, bool resident) {
  std::lock_guard<std::mutex> lk(req_mu_);
  Layer& L = layers_[id];
  L.seeded = resident;
  for (auto& s : L.st) s = resident ? 2 : 0;
}

void PlannedEngine::set_source_packed(LayerID id, bool packed) {
  std::lock_guard<std::mutex> lk(req_mu_);
  layers_[id].src_packed = packed;
}

std::vector<int64_t> PlannedEngine::resident_chunks(LayerID id) {
  std::lock_guard<std::mutex> lk(req_mu_);
  std::vector<int64_t> out;
  auto it = layers_.find(id);
  if (it == layers_.end()) return out;
  for (size_t c = 0; c < it->second.st.size(); ++c)
    if (it->second.st[c] == 2) out.push_back(int64_t(c));
  return out;
}

std::map<LayerID, CrcManifest> PlannedEngine::manifest() {
  std::lock_guard<std::mutex> lk(req_mu_);
  std::map<LayerID, CrcManifest> out;
  for (auto& kv : layers_)
    if (!kv.second.manifest.crc.empty()) out[kv.first] = kv.second.manifest;
  return out;
}

PlannedStats PlannedEngine::stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return stats_;
}

std::string PlannedEngine::error() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return error_;
}

void PlannedEngine::fail(const std::string& what) {
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    if (error_.empty()) error_ = what;
  }
  failed_ = true;
  log::error(int64_t(self_node_)).s("error", what).msg("data engine failure");
  idle_cv_.notify_all();
}

// ------------------------------------------------------------ DataEngine

bool PlannedEngine::on_message(const MessagePtr& m) {
  if (m->type != MsgType::XferBatch && m->type != MsgType::Shrink) return false;
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    if (m->type == MsgType::Shrink) {
      Req r{Req::Shrink, {}, 0, 0, 0};
      r.dead = m->peers;
      r.generation = m->seq;
      r.comm_id = m->payload_str;
      reqs_.push_back(std::move(r));
    } else {
      Req r{Req::Batch, m->jobs, 0, 0, 0};
      r.order = m->order;
      reqs_.push_back(std::move(r));
    }
    busy_ = true;
  }
  req_cv_.notify_all();
  return true;
}

void PlannedEngine::send_range(NodeID dest, LayerID layer_id, int64_t, int64_t, int64_t, int64_t) {
  log::error(int64_t(self_node_)).u("layer", layer_id).u("dest", dest)
      .msg("planned engine: sends are scheduled by the leader's XferBatch, not pushed");
}

void PlannedEngine::load_range(LayerID layer_id, int64_t offset, int64_t size, int64_t, int64_t) {
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    reqs_.push_back(Req{Req::Load, {}, layer_id, offset, size});
    busy_ = true;
  }
  req_cv_.notify_all();
}

void PlannedEngine::host_prefix_ready(LayerID layer_id, const uint8_t* base, int64_t prefix, int64_t total) {
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    Req r{Req::HostReady, {}, layer_id, prefix, total};
    r.base = base;
    reqs_.push_back(std::move(r));
    busy_ = true;
  }
  req_cv_.notify_all();
}

void PlannedEngine::quiesce() {
  std::unique_lock<std::mutex> lk(req_mu_);
  // Bounded: a transfer whose peer died must not hang the caller forever.
  bool ok = cv_wait_for(idle_cv_, lk, 120.0, [&] {
    return (reqs_.empty() && !busy_) || failed_.load() || stopped_.load();
  });
  if (!ok) log::error(int64_t(self_node_)).msg("quiesce timed out: data plane still busy");
}

void PlannedEngine::reset_session() {
  quiesce();
  uint64_t want;
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    want = resets_done_ + 1;
    reqs_.push_back(Req{Req::Reset, {}, 0, 0, 0});
    busy_ = true;
  }
  req_cv_.notify_all();
  {
    std::unique_lock<std::mutex> lk(req_mu_);
    idle_cv_.wait(lk, [&] { return resets_done_ >= want || failed_.load() || stopped_.load(); });
  }
  if (failed_) throw std::runtime_error("data engine failed: " + error());
}

std::vector<ProbeOp> PlannedEngine::probe(const std::vector<ProbeOp>& ops, double timeout_s) {
  quiesce();
  ProbeJob job;
  job.ops = ops;
  job.timeout_s = timeout_s;
  {
    std::lock_guard<std::mutex> lk(req_mu_);
    Req r{Req::Probe, {}, 0, 0, 0};
    r.probe = &job;
    reqs_.push_back(std::move(r));
    busy_ = true;
  }
  req_cv_.notify_all();
  {
    std::unique_lock<std::mutex> lk(req_mu_);
    idle_cv_.wait(lk, [&] { return job.finished || failed_.load() || stopped_.load(); });
    if (!job.finished) throw std::runtime_error("probe: data engine stopped: " + error());
  }
  return job.ops;
}

void PlannedEngine::run_probe(ProbeJob& job) {
  trace::Scoped tr("dissem.probe");
  int64_t maxb = 0;
  std::map<int, std::vector<size_t>> by_lane;
  for (size_t i = 0; i < job.ops.size(); ++i) {
    ProbeOp& o = job.ops[i];
    if (o.peer < 0 || o.peer >= cfg_.world || o.peer == cfg_.rank || o.bytes <= 0)
      throw std::runtime_error("probe: bad op (peer " + std::to_string(o.peer) + ")");
    o.lane = lane_for(o.peer, o.send);
    by_lane[o.lane].push_back(i);
    maxb = std::max(maxb, o.bytes);
  }
  // One send buffer read by every send; one landing buffer per recv.
  std::vector<uint8_t*> bufs;
  uint8_t* sbuf = backend_->alloc(maxb);
  bufs.push_back(sbuf);
  struct G {
    Ev ev;
    std::vector<size_t> ops;
    bool done = false;
  };
  std::vector<G> groups;
  const double t0 = vclock::now();
  for (auto& kv : by_lane) {
    std::vector<XOp> xops;
    for (size_t i : kv.second) {
      const ProbeOp& o = job.ops[i];
      uint8_t* p = sbuf;
      if (!o.send) {
        p = backend_->alloc(o.bytes);
        bufs.push_back(p);
      }
      xops.push_back(XOp{o.send, o.peer, p, o.bytes});
    }
    CallMark cm(this, "probe", kv.first);
    groups.push_back(G{backend_->group(xops, {}, kv.first), kv.second});
  }
  size_t left = groups.size();
  while (left > 0) {
    const double now = vclock::now();
    for (auto& g : groups) {
      if (g.done) continue;
      const int r = backend_->query(g.ev);
      if (r == 0) continue;
      g.done = true;
      --left;
      double ms = r > 0 ? backend_->group_ms(g.ev) : -1;
      if (r > 0 && ms < 0) ms = (now - t0) * 1e3;
      for (size_t i : g.ops) {
        job.ops[i].done = r > 0;
        job.ops[i].ms = ms;
      }
      backend_->release(g.ev);
    }
    if (left == 0 || now - t0 > job.timeout_s) break;
    vclock::sleep_for(200e-6);
  }
  if (left == 0) {
    for (uint8_t* b : bufs) backend_->free(b);
  } else {
    log::error(int64_t(self_node_)).i("stalled_groups", int64_t(left)).f("timeout_s", job.timeout_s)
        .msg("link probe: lanes did not complete");
  }
}

// ------------------------------------------------------------ issue thread

uint32_t PlannedEngine::crc_slot() {
  uint32_t s = crc_next_;
  crc_next_ = (crc_next_ + 1) % kCrcSlots;
  return s;
}

void PlannedEngine::ev_drop(Ev e) {
  if (!e) return;
  auto it = evref_.find(e);
  if (it == evref_.end() || --it->second <= 0) {
    if (it != evref_.end()) evref_.erase(it);
    backend_->release(e);
  }
}

void PlannedEngine::set_chunk_ev(Layer& L, int64_t c, Ev e) {
  Ev& slot = L.ev[size_t(c)];
  if (slot == e) return;
  ev_hold(e);
  ev_drop(slot);
  slot = e;
}

// Non-blocking token bucket with one chunk of burst: a chunk may go when the
// bucket is full enough for it; tokens may go negative, so the long-run rate
// is exactly `rate`.
bool PlannedEngine::pace_ready(uint64_t key, int64_t rate, int64_t n) {
  if (rate <= 0) return true;
  const double now = vclock::now();
  Pace& p = pace_[key];
  // Mode-3 job buckets hold two chunks: the plan runs every link at exactly its
  // capacity (size/T per job), so a job held back behind staging or its lane
  // must be able to catch up by a chunk, or the lost time adds to T for good
  // (sim at N = 8: 273 -> 237 ms against a planned 215). Link and tier caps
  // keep one chunk, like x/time/rate's initial burst.
  const double cap = double(n) * ((key >> 62) == 1 ? 2.0 : 1.0);
  if (p.rate <= 0) {
    p.rate = double(rate);
    p.burst = cap;
    p.tokens = double(n);
    p.last = now;
  }
  p.rate = double(rate);
  p.burst = std::max(p.burst, cap);
  p.tokens = std::min(p.burst, p.tokens + (now - p.last) * p.rate);
  p.last = now;
  return p.tokens >= double(n) - 0.5;
}

void PlannedEngine::pace_take(uint64_t key, int64_t rate, int64_t n) {
  if (rate > 0) pace_[key].tokens -= double(n);
}

void PlannedEngine::add_batch(std::vector<XferJob>& jobs, uint8_t order) {
  std::sort(jobs.begin(), jobs.end(), [](const XferJob& a, const XferJob& b) { return a.seq < b.seq; });
  std::vector<Piece> pieces;
  const int64_t cb = grid_;
  const uint64_t batch = ++batches_;
  for (auto& j : jobs) {
    Kind kind;
    int peer;
    const bool bcast = j.dst == kAllRanks;
    if (bcast) {
      kind = j.src == self_node_ ? Kind::Send : Kind::Recv;
      peer = rank_of(j.src);
    } else if (j.src == self_node_ && j.dst == self_node_) {
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
    for (int64_t pos = j.offset; pos < end;) {
      const int64_t c = pos / cb;
      const int64_t cend = std::min((c + 1) * cb, L.size);
      const int64_t e = std::min(cend, end);
      // Ordering key (batch, chunk index in the layer, seq): a relay of chunk c
      // (a later phase, so a larger seq) always sorts after the recv of chunk c
      // it forwards, whatever byte ranges the two jobs cover.
      // Job-major batches (mode 2) order a lane job by job instead (pidx =
      // seq, then chunk): a sender's pull jobs start as acks return, so its
      // lanes hold different layers, and chunk-major order would interleave
      // them - a lane waiting on layer B's chunk 0 while the copy queue stages
      // layer A for the others (sim, N = 8: 224 -> 216 ms, bound 214.7).
      const int64_t pidx = order == 1 ? int64_t((j.seq << 24) | uint64_t(c)) : c;
      Piece p{kind, j.seq, pidx, peer, j.layer, pos, e - pos, L.size, c, pos == c * cb && e == cend};
      p.src_node = j.src;
      p.bcast = bcast;
      p.rate = j.rate;
      p.batch = batch;
      // Collectives run on lane 0 (every rank's copy of the lane-0 communicator).
      p.lane = bcast || kind == Kind::Local ? 0 : lane_for(peer, kind == Kind::Send);
      const int64_t ci = c - first_chunk;
      if (ci < int64_t(j.crc.size())) {
        // a partial piece carries its chunk's CRC for the check once every
        // piece of the chunk has landed (partial_landed)
        (p.full ? p.has_crc : p.has_ccrc) = true;
        (p.full ? p.crc : p.ccrc) = j.crc[size_t(ci)];
        if (p.full && kind != Kind::Recv) L.job_crc[c] = p.crc;  // staging checks it without a manifest
      }
      pieces.push_back(p);
      pos = e;
    }
  }
  std::stable_sort(pieces.begin(), pieces.end(), [](const Piece& a, const Piece& b) {
    return a.pidx != b.pidx ? a.pidx < b.pidx : a.seq < b.seq;
  });
  for (auto& p : pieces) {
    if (p.kind == Kind::Local) continue;
    if (p.kind == Kind::Send && !p.bcast) fwd_pending_[{p.layer, p.chunk}].insert(key_of(p));
    ops_[size_t(p.lane)].push_back(p);
  }
  for (auto& p : pieces) {
    if (p.kind != Kind::Local) continue;
    // Local promotions take no part in the P2P order. A chunk this rank also
    // sends is staged when its first send needs it (the lanes' key order), so
    // a promotion never queues a layer on the copy queue ahead of the chunks
    // the links are waiting for (mode 2 at N = 8: a self-load of the layer
    // being sent staged all 16 chunks at once and the lanes' next layer
    // waited ~17 ms behind them). Any other chunk stages right away, so PCIe
    // runs ahead of the xGMI rounds that forward the same chunks.
    // While this rank has sends queued, other promotions trickle in at most
    // kPromoteAhead chunks at a time (issue_some) instead of queueing whole
    // layers ahead of the sends' chunks.
    Layer& L = layer(p.layer);
    if (L.st[size_t(p.chunk)] == 0 && !fwd_pending_.empty()) {
      L.want[size_t(p.chunk)] = 1;
      deferred_local_.push_back({p.layer, p.chunk});
      continue;
    }
    if (ensure_chunk(L, p.layer, p.chunk, true) < 0) fail("no source to load layer " + std::to_string(p.layer));
  }
  int64_t ns = 0, nr = 0;
  for (auto& p : pieces) (p.kind == Kind::Send ? ns : nr) += p.kind == Kind::Local ? 0 : 1;
  log::info(int64_t(self_node_)).u("batch", batch).i("jobs", int64_t(jobs.size())).i("sends", ns).i("recvs", nr)
      .msg("transfer batch queued");
}

bool PlannedEngine::issue_some() {
  if (recovering_ || dead_) return false;
  // Promotions left to a send whose staging they would share: once the send
  // staged the chunk (or no longer will: cancelled by a re-plan) they are done
  // (the chunk's check reports it landed, L.want) or staged here.
  for (auto it = promoting_.begin(); it != promoting_.end();)
    it = layers_[it->first].st[size_t(it->second)] == 1 ? std::next(it) : promoting_.erase(it);
  for (size_t n = deferred_local_.size(); n > 0 && !failed_; --n) {
    auto lc = deferred_local_.front();
    deferred_local_.pop_front();
    Layer& L = layers_[lc.first];
    if (L.st[size_t(lc.second)] != 0) continue;
    if (fwd_pending_.count(lc) || (!fwd_pending_.empty() && promoting_.size() >= size_t(kPromoteAhead))) {
      deferred_local_.push_back(lc);
      continue;
    }
    if (ensure_chunk(L, lc.first, lc.second, true) < 0) fail("no source to load layer " + std::to_string(lc.first));
    if (L.st[size_t(lc.second)] == 1) promoting_.insert(lc);
  }
  // Local promotions held back by tier pacing.
  for (size_t n = local_wait_.size(); n > 0 && !failed_; --n) {
    auto lc = local_wait_.front();
    local_wait_.pop_front();
    Layer& L = layers_[lc.first];
    if (L.st[size_t(lc.second)] == 0 && ensure_chunk(L, lc.first, lc.second, true) < 0)
      fail("no source to load layer " + std::to_string(lc.first));
  }
  // Lanes are independent: a lane whose next piece cannot go yet (data not
  // staged or received, pacing, in-flight cap) does not hold the others.
  bool progress = false;
  for (int lane = 0; lane < lanes_; ++lane) progress |= issue_lane(lane);
  flush_checks();  // the chunks this pass's groups land (and staged): batched checks
  return progress;
}

bool PlannedEngine::issue_lane(int lane) {
  bool progress = false;
  auto& q = ops_[size_t(lane)];
  auto& infl = inflight_[size_t(lane)];
  const double now = vclock::now();
  const int cap = std::max(4, cfg_.max_inflight_groups / lanes_);
  while (!q.empty() && int(infl.size()) < cap && !failed_) {
    std::vector<Piece> group;
    std::map<int, int> nsend, nrecv;
    std::set<std::pair<LayerID, int64_t>> recv_chunks;
    std::vector<std::pair<uint64_t, std::pair<int64_t, int64_t>>> takes;  // pacing: key, (rate, bytes)
    size_t take = 0;
    for (; take < q.size(); ++take) {
      Piece& p = q[take];
      if (p.bcast) {
        // A collective runs in a group of its own (every rank reaches it at the
        // same key, so the ordering argument above covers it too).
        if (!group.empty()) break;
        if (p.kind == Kind::Send && ensure_chunk(layer(p.layer), p.layer, p.chunk, false) <= 0) break;
        group.push_back(p);
        ++take;
        break;
      }
      if (p.kind == Kind::Send) {
        if (nsend[p.peer] >= cfg_.group_peers) break;
        if (recv_chunks.count({p.layer, p.chunk})) break;  // forward only after its recv is posted
        Layer& L = layer(p.layer);
        if (ensure_chunk(L, p.layer, p.chunk, false) <= 0) break;  // not staged / received yet (or paced)
        // Pacing: the job's rate (mode 3) and the link cap to this peer.
        int64_t link = 0;
        if (!cfg_.link_rate.empty()) {
          auto it = cfg_.link_rate.find(cfg_.rank_nodes[size_t(p.peer)]);
          if (it != cfg_.link_rate.end()) link = it->second;
        }
        const uint64_t kj = kPaceJob | p.seq, kp = kPacePeer | uint64_t(p.peer);
        if (!pace_ready(kj, p.rate, p.len) || !pace_ready(kp, link, p.len)) {
          std::lock_guard<std::mutex> lk(stats_mu_);
          stats_.paced++;
          break;
        }
        takes.push_back({kj, {p.rate, p.len}});
        takes.push_back({kp, {link, p.len}});
        nsend[p.peer]++;
        group.push_back(p);
        continue;
      }
      if (nrecv[p.peer] >= cfg_.group_peers) break;
      if (!p.bcast) {
        // Crossing jobs (both ends hold the layer, e.g. mode-2 steals): this
        // rank also sends the chunk, with a smaller key, on another lane. Post
        // that send first - it stages from the local source - so it never
        // waits on this recv's mark (a larger key; see the argument above).
        auto f = fwd_pending_.find({p.layer, p.chunk});
        if (f != fwd_pending_.end() && !f->second.empty() && *f->second.begin() < key_of(p) &&
            has_local_source(layer(p.layer), p.layer, p.chunk))
          break;
      }
      nrecv[p.peer]++;
      recv_chunks.insert({p.layer, p.chunk});
      group.push_back(p);
      // Lanes: a chunk that this rank forwards on (possibly) another lane is
      // released to that send by a mark behind this group - close the group
      // here so the mark never waits on pieces with larger keys.
      if (lanes_ > 1) {
        auto f = fwd_pending_.find({p.layer, p.chunk});
        if (f != fwd_pending_.end() && !f->second.empty()) {
          ++take;
          break;
        }
      }
    }
    if (group.empty()) break;
    for (auto& t : takes) pace_take(t.first, t.second.first, t.second.second);
    q.erase(q.begin(), q.begin() + int64_t(take));
    trace::Scoped tr(group.front().bcast ? "dissem.bcast" : "dissem.p2p_group");
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<Ev> waits;
    std::vector<XOp> xops;
    int64_t sent = 0, recvd = 0;
    for (auto& p : group) {
      Layer& L = layers_[p.layer];
      if (!L.dev) L.dev = backend_->alloc(L.size);
      if (p.kind == Kind::Send) {
        if (L.st[size_t(p.chunk)] == 1 && L.rkey[size_t(p.chunk)] > key_of(p)) {
          std::lock_guard<std::mutex> lk(stats_mu_);
          if (stats_.order_violations++ == 0)
            log::error(int64_t(self_node_)).u("layer", p.layer).i("chunk", p.chunk)
                .msg("send waits on a recv with a larger key (deadlock-prone order)");
        }
        if (L.st[size_t(p.chunk)] == 1 && L.ev[size_t(p.chunk)]) {
          Ev e = L.ev[size_t(p.chunk)];
          if (std::find(waits.begin(), waits.end(), e) == waits.end()) waits.push_back(e);
        }
        if (!p.bcast) {
          auto f = fwd_pending_.find({p.layer, p.chunk});
          if (f != fwd_pending_.end()) {
            auto k = f->second.find(key_of(p));
            if (k != f->second.end()) f->second.erase(k);
            if (f->second.empty()) fwd_pending_.erase(f);
          }
        }
        sent += p.len;
      } else {
        recvd += p.len;
      }
      uint8_t* at = L.dev + p.off;
      if (p.kind == Kind::Recv && !p.bcast && p.full) {
        // A chunk this rank stages (or reads from disk), or already holds: a
        // mode-2 steal of a dest's own load, a re-dispatch. The peer's copy
        // lands beside it, is checked there and dropped - the live slot keeps
        // exactly one writer.
        const uint8_t s = L.st[size_t(p.chunk)];
        if (s == 1 || s == 2 || s == 3) {
          p.scratch = scratch_take();
          at = p.scratch;
        }
      }
      xops.push_back(XOp{p.kind == Kind::Send, p.peer, at, p.len, p.bcast});
    }
    Ev g;
    {
      CallMark cm(this, "group", lane);
      g = backend_->group(xops, waits, lane);
    }
    Inflight inf{g, now, {}, {}};
    for (auto& p : group) {
      if (std::find(inf.peers.begin(), inf.peers.end(), p.peer) == inf.peers.end()) inf.peers.push_back(p.peer);
      if (p.kind == Kind::Send && !p.bcast &&
          std::find(inf.send_peers.begin(), inf.send_peers.end(), p.peer) == inf.send_peers.end())
        inf.send_peers.push_back(p.peer);
      if (p.kind == Kind::Recv && !p.bcast &&
          std::find(inf.recv_peers.begin(), inf.recv_peers.end(), p.peer) == inf.recv_peers.end())
        inf.recv_peers.push_back(p.peer);
    }
    infl.push_back(std::move(inf));
    // Fault injection: damage some received chunks behind the group, before their check.
    Ev landed_ev = g;
    int64_t injected = 0;
    if (cfg_.inject_corrupt > 0) {
      std::uniform_real_distribution<double> u(0.0, 1.0);
      for (auto& p : group) {
        if (p.kind != Kind::Recv || p.len < 4 || u(inject_rng_) >= cfg_.inject_corrupt) continue;
        Ev c = backend_->corrupt(p.scratch ? p.scratch : layers_[p.layer].dev + p.off, lane);
        if (landed_ev != g) backend_->release(landed_ev);
        landed_ev = c;
        injected++;
      }
    }
    // Receivers: chunks are valid behind `g` on this lane; check them on the
    // verify queue. With one lane a later send of the chunk is ordered behind
    // `g` on the same queue; with several, it waits for a mark on this lane.
    Ev mark = 0;
    for (auto& p : group) {
      if (p.kind != Kind::Recv) continue;
      Layer& L = layers_[p.layer];
      if (p.scratch) {
        // the chunk's state stays its staging's; only the peer's copy is checked
        PendingCheck pc;
        pc.piece = p;
        pc.wait = landed_ev;
        if (cfg_.verify && p.has_crc) {
          pc.slot = crc_slot();
          pc.req = Backend::CheckReq{p.scratch, p.len, pc.slot};
          pc.has_req = true;
        }
        pending_reqs_ += pc.has_req ? 1 : 0;
        pending_checks_.push_back(pc);
        continue;
      }
      L.st[size_t(p.chunk)] = 1;
      L.rkey[size_t(p.chunk)] = key_of(p);
      if (lanes_ > 1 && !p.bcast) {
        if (!mark) {
          CallMark cm(this, "mark", lane);
          mark = backend_->mark(lane);
        }
        set_chunk_ev(L, p.chunk, mark);
      } else {
        set_chunk_ev(L, p.chunk, 0);  // pending on the comm queue itself: later sends are ordered behind it
      }
      // The chunk's check joins the pending batch behind this group's landing
      // (flush_checks at the end of the issue pass): the chunks every lane
      // landed in one pass share verify launches.
      PendingCheck pc;
      pc.piece = p;
      pc.wait = landed_ev;  // alive until the flush: the group is polled after it
      if (cfg_.unpack_store && p.full) {
        // fused check + dequantization of the landed packed chunk
        const uint32_t s = crc_slot();
        pc.req = unpack_req(L, p.chunk, s);
        pc.has_req = true;
        if (cfg_.verify && p.has_crc) pc.slot = s;
      } else if (cfg_.verify && p.has_crc && p.full) {
        pc.slot = crc_slot();
        pc.req = Backend::CheckReq{L.dev + p.off, p.len, pc.slot};
        pc.has_req = true;
      }
      pending_reqs_ += pc.has_req ? 1 : 0;
      pending_checks_.push_back(pc);
    }
    if (landed_ev != g) owned_waits_.push_back(landed_ev);  // released after the flush
    {
      std::lock_guard<std::mutex> lk(stats_mu_);
      stats_.groups++;
      stats_.pieces += int64_t(group.size());
      stats_.bytes_sent += sent;
      stats_.bytes_recv += recvd;
      stats_.injected += injected;
      for (auto& p : group) (p.kind == Kind::Send ? stats_.peer_sent : stats_.peer_recv)[p.peer] += p.len;
      stats_.issue_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    progress = true;
    if (cfg_.inject_die_after_groups > 0 && ++groups_issued_ >= cfg_.inject_die_after_groups) {
      die();
      break;
    }
  }
  return progress;
}

void PlannedEngine::poll() {
  flush_checks();  // what was staged since the issue pass: batched checks
  const double now = vclock::now();
  for (int lane = 0; lane < lanes_; ++lane) {
    auto& infl = inflight_[size_t(lane)];
    while (!infl.empty()) {
      Inflight& head = infl.front();
      int r = backend_->query(head.ev);
      if (r == 0) {
        // Watchdog: a group whose partner never posts (dead or hung peer) would
        // block its lane forever. Report the in-flight peers to the leader
        // (which probes them and shrinks the communicator around a dead one);
        // fail if nothing resolves it.
        double age = now - head.t0;
        if (node_ && cfg_.suspect_s > 0 && age > cfg_.suspect_s && now - last_suspect_ > std::max(cfg_.suspect_s, 1.0)) {
          // Not (yet) a failure: if the peers are alive the group may still
          // complete. Name every in-flight peer: the group at the head may be
          // waiting on a live rank that itself waits on the dead one.
          last_suspect_ = now;
          suspect(inflight_peers(), "P2P group pending for " + std::to_string(int(age)) + " s", false);
        }
        if (cfg_.group_timeout_s > 0 && age > cfg_.group_timeout_s)
          fail("P2P group pending for " + std::to_string(int(age)) + " s: a peer rank is dead or stuck");
        break;
      }
      if (r < 0) {
        if (!node_) {
          fail("P2P group failed: " + backend_->async_error());
          return;
        }
        // The communicator is broken (e.g. a peer's connection died): stop and
        // let the leader decide; its Shrink resets everything in flight.
        if (!recovering_) suspect(inflight_peers(), "P2P group failed: " + backend_->async_error(), true);
        break;
      }
      const double ms = backend_->group_ms(head.ev);
      {
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.group_us_hist[log2_bucket(head.t0)]++;
        if (ms >= 0) {
          stats_.lane_busy_ms[size_t(lane)] += ms;
          for (int p : head.peers) stats_.peer_busy_ms[p] += ms;
          for (int p : head.send_peers) stats_.peer_send_busy_ms[p] += ms;
          for (int p : head.recv_peers) stats_.peer_recv_busy_ms[p] += ms;
        }
      }
      backend_->release(head.ev);
      infl.pop_front();
      ++completions_;
    }
    if (failed_ || recovering_) break;
  }
  std::vector<Verify> followups;  // whole-chunk checks of chunks completed by partial pieces
  for (auto it = verifies_.begin(); it != verifies_.end();) {
    int r = backend_->query(it->ev);
    if (r == 0) {
      ++it;
      continue;
    }
    if (r < 0) {
      if (node_) {  // behind a failed group: the leader's Shrink resets it
        if (!recovering_) suspect(inflight_peers(), "landing failed: " + backend_->async_error(), true);
        break;
      }
      fail("landing failed: " + backend_->async_error());
      return;
    }
    for (size_t i = 0; i < it->pieces.size(); ++i) {
      const Piece& p = it->pieces[i];
      Layer& L = layers_[p.layer];
      if (p.scratch) {
        const bool bad = it->slots[i] != ~0u && backend_->crc_result(it->slots[i]) != p.crc;
        scratch_free_.push_back(p.scratch);  // its check has completed
        {
          std::lock_guard<std::mutex> lk(stats_mu_);
          stats_.scratch_landings++;
          stats_.verify_failures += bad ? 1 : 0;  // the peer's copy; the local one stands
        }
        // landed for the leader once the local copy is resident (its staging's check)
        if (L.st[size_t(p.chunk)] == 2) landed(p);
        else L.want[size_t(p.chunk)] = 1;
        continue;
      }
      if (it->slots[i] != ~0u) {
        uint32_t got = backend_->crc_result(it->slots[i]);
        if (got != p.crc) {
          nack(p, L, got);
          if (failed_) return;
          continue;
        }
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.bytes_verified += p.len;
      } else if (p.kind == Kind::Recv && !p.full) {
        // Part of a chunk (e.g. two relays split it): it is checked, and
        // reported landed, as a whole once all of its bytes are here.
        partial_landed(L, p, followups);
        continue;
      } else if (p.kind == Kind::Recv) {
        std::lock_guard<std::mutex> lk(stats_mu_);
        stats_.unverified_pieces++;
      }
      if (p.full) L.st[size_t(p.chunk)] = 2;
      set_chunk_ev(L, p.chunk, 0);
      if (p.kind == Kind::Recv) {
        landed(p);
      } else if (L.want[size_t(p.chunk)]) {
        landed(p);
        L.want[size_t(p.chunk)] = 0;
      }
    }
    {
      const double vms = backend_->group_ms(it->ev);
      std::lock_guard<std::mutex> lk(stats_mu_);
      stats_.land_us_hist[log2_bucket(it->t0)] += int64_t(it->pieces.size());
      if (vms > 0) stats_.verify_busy_ms += vms;
    }
    backend_->release(it->ev);
    it = verifies_.erase(it);
  }
  for (auto& v : followups) verifies_.push_back(std::move(v));
  std::vector<std::pair<LayerID, int64_t>> again;
  again.swap(restage_);
  for (auto& lc : again) {
    Layer& L = layers_[lc.first];
    L.st[size_t(lc.second)] = 0;
    stage_chunk(L, lc.first, lc.second);
  }
}

void PlannedEngine::take_requests(bool block) {
  std::deque<Req> got;
  {
    std::unique_lock<std::mutex> lk(req_mu_);
    if (block && reqs_.empty() && !stop_req_) {
      busy_ = false;
      idle_cv_.notify_all();
      cv_wait_for(req_cv_, lk, 0.05, [&] { return !reqs_.empty() || stop_req_.load(); });
    }
    got.swap(reqs_);
    if (!got.empty()) busy_ = true;
  }
  for (auto& r : got) {
    switch (r.type) {
      case Req::Batch:
        add_batch(r.jobs, r.order);
        break;
      case Req::Load: {
        Layer& L = layer(r.layer);
        if (!L.size) break;
        for (int64_t c = r.off / grid_; c * grid_ < r.off + r.len && c < int64_t(L.st.size()); ++c)
          if (ensure_chunk(L, r.layer, c, true) < 0) fail("no source to load layer " + std::to_string(r.layer));
        break;
      }
      case Req::Reset: {
        for (auto& kv : layers_) {
          Layer& L = kv.second;
          for (size_t c = 0; c < L.st.size(); ++c) {
            L.st[c] = L.seeded ? 2 : 0;
            set_chunk_ev(L, int64_t(c), 0);
            L.want[c] = 0;
            L.fails[c] = 0;
          }
          L.host = nullptr;  // re-read the source from the next session's store
          L.host_prefix = -1;
          L.client_requested = false;
          L.stage_rate = -1;
          L.ranges_known = false;
          L.part.clear();
          if (cfg_.poison && !L.seeded && L.dev) backend_->zero_sync(L.dev, L.size);
        }
        pace_.clear();
        local_wait_.clear();
        deferred_local_.clear();
        promoting_.clear();
        fwd_pending_.clear();
        std::lock_guard<std::mutex> lk(req_mu_);
        resets_done_++;
        idle_cv_.notify_all();
        break;
      }
      case Req::Shrink:
        do_shrink(r.dead, r.generation, r.comm_id);
        break;
      case Req::HostReady: {
        Layer& L = layer(r.layer);
        if (!L.size || !r.base) break;
        L.host = r.base;
        L.path.clear();
        const int64_t src_total = r.len;
        L.host_prefix = r.off >= src_total ? -1 : r.off;
        // Stage what this rank itself needs now; sends pick theirs up on their next pass.
        for (int64_t c = 0; c < int64_t(L.st.size()); ++c) {
          if (L.host_prefix >= 0 && c * src_grid(L) + src_len(L, c) > L.host_prefix) break;
          if (L.want[size_t(c)] && L.st[size_t(c)] == 0 && ensure_chunk(L, r.layer, c, true) < 0)
            fail("no source to load layer " + std::to_string(r.layer));
        }
        break;
      }
      case Req::Probe: {
        try {
          run_probe(*r.probe);
        } catch (const std::exception& e) {
          fail(std::string("probe: ") + e.what());
        }
        std::lock_guard<std::mutex> lk(req_mu_);
        r.probe->finished = true;
        idle_cv_.notify_all();
        break;
      }
      case Req::Stop:
        break;
    }
  }
}

void PlannedEngine::run() {
  try {
    backend_->init_thread();
    double last_async_check = vclock::now();
    while (!stop_req_) {
      take_requests(idle());
      if (stop_req_) break;
      if (failed_) {
        // Drop queued work; in-flight P2P ops are aborted at shutdown.
        for (auto& q : ops_) q.clear();
        for (auto& q : inflight_) q.clear();
        verifies_.clear();
        drop_pending_checks();
        local_wait_.clear();
        deferred_local_.clear();
        promoting_.clear();
        std::lock_guard<std::mutex> lk(req_mu_);
        busy_ = false;
        idle_cv_.notify_all();
        continue;
      }
      if (dead_) {
        // Fault injection: a crashed rank does nothing until shutdown.
        std::lock_guard<std::mutex> lk(req_mu_);
        reqs_.clear();
        busy_ = false;
        idle_cv_.notify_all();
        vclock::sleep_for(0.005);
        continue;
      }
      loop_ticks_.fetch_add(1, std::memory_order_relaxed);
      idle_flag_ = idle();
      pump_disk();
      bool progress = issue_some();
      poll();
      if (recovering_ && cfg_.group_timeout_s > 0 &&
          vclock::now() - recover_since_ > cfg_.group_timeout_s)
        fail("data plane stalled and the leader did not shrink the communicator");
      {
        std::lock_guard<std::mutex> lk(req_mu_);
        busy_ = !idle() || !reqs_.empty();
        if (!busy_) idle_cv_.notify_all();
      }
      const double now = vclock::now();
      if (now - last_async_check > 0.1) {
        last_async_check = now;
        std::string e = backend_->async_error();
        if (!e.empty() && !recovering_) {
          if (node_) {
            suspect(inflight_peers(), "async error: " + e, true);
          } else {
            fail("async error: " + e);
          }
        }
      }
      // A quiet data plane with work left (nothing issued or completed for
      // suspect_s): say what every lane waits for - also on ranks whose lanes
      // hold no old group, which the suspect report above never covers.
      if (progress || completions_ != quiet_mark_ || idle()) {
        quiet_mark_ = completions_;
        quiet_since_ = now;
      } else if (cfg_.suspect_s > 0 && now - quiet_since_ > cfg_.suspect_s) {
        quiet_since_ = now;
        log::warn(int64_t(self_node_)).s("state", describe_stall()).f("quiet_s", cfg_.suspect_s)
            .msg("data plane waiting: no group issued or completed");
      }
      if (!progress && !idle()) vclock::sleep_for(20e-6);
    }
  } catch (const std::exception& e) {
    fail(e.what());
  }
  std::lock_guard<std::mutex> lk(req_mu_);
  busy_ = false;
  idle_cv_.notify_all();
}

}  // namespace dissem
