// Planned engine (planned_engine.h), the local side of a chunk: staging from
// host memory or the disk tier (O_DIRECT readers into pinned bounce buffers,
// then H2D on the copy queues, fp8 packing on the way), tier pacing, and the
// checks of staged and landed chunks - batched onto the verify queue
// (flush_checks) - with their outcome: landed, partial coverage, NACK.
#include "engine/planned_engine.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "core/fp8.h"
#include "core/log.h"
#include "core/trace.h"
#include "roles/node.h"

namespace dissem {

bool PlannedEngine::stage_paced(Layer& L, LayerID id, int64_t c) {
  if (L.stage_rate < 0) {
    LayerSrc src;
    L.stage_rate = 0;
    if (node_ && node_->store().get(id, &src)) {
      L.stage_rate = std::max<int64_t>(0, src.meta.limit_rate);
      L.stage_tier = int(src.meta.source_type);
    }
  }
  if (L.stage_rate <= 0) return false;
  const uint64_t key = kPaceTier | uint64_t(L.stage_tier);
  const int64_t n = src_len(L, c);
  if (!pace_ready(key, L.stage_rate, n)) {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.paced++;
    return true;
  }
  pace_take(key, L.stage_rate, n);
  return false;
}

Backend::CheckReq PlannedEngine::unpack_req(Layer& L, int64_t c, uint32_t slot) {
  const int64_t src_total = fp8::source_size(L.size, cfg_.chunk_bytes, cfg_.pack_block);
  if (!L.out) L.out = backend_->alloc(src_total);
  const int64_t slen = std::min(cfg_.chunk_bytes, src_total - c * cfg_.chunk_bytes);
  return Backend::CheckReq{L.dev + c * grid_, slen, slot, L.out + c * cfg_.chunk_bytes, cfg_.pack_block};
}

void PlannedEngine::partial_landed(Layer& L, const Piece& p, std::vector<Verify>& out) {
  PartChunk& pc = L.part[p.chunk];
  pc.got.add(p.off, p.off + p.len);
  if (p.has_ccrc) {
    pc.has_crc = true;
    pc.crc = p.ccrc;
  }
  const int64_t a = p.chunk * grid_, b = std::min(a + grid_, L.size);
  if (!pc.got.contains(a, b)) return;
  Piece f = p;
  f.off = a;
  f.len = b - a;
  f.full = true;
  f.has_crc = cfg_.verify && pc.has_crc;
  f.crc = pc.crc;
  L.part.erase(p.chunk);
  Verify v;
  uint32_t slot = ~0u;
  std::vector<Backend::CheckReq> reqs;
  if (cfg_.unpack_store) {
    const uint32_t s = crc_slot();
    reqs.push_back(unpack_req(L, f.chunk, s));
    reqs.back().expect = f.crc;
    if (f.has_crc) slot = s;
  } else if (f.has_crc) {
    slot = crc_slot();
    reqs.push_back(Backend::CheckReq{L.dev + a, b - a, slot});
    reqs.back().expect = f.crc;
  }
  v.ev = backend_->verify(reqs, {});
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.verify_calls++;
    stats_.verify_chunks += int64_t(reqs.size());
  }
  v.pieces.push_back(f);
  v.slots.push_back(slot);
  out.push_back(std::move(v));
}

void PlannedEngine::landed(const Piece& p) {
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

void PlannedEngine::nack(const Piece& p, Layer& L, uint32_t got) {
  const size_t c = size_t(p.chunk);
  char buf[200];
  snprintf(buf, sizeof buf, "CRC32C mismatch layer %llu chunk %lld from node %llu: got %08x want %08x",
           (unsigned long long)p.layer, (long long)p.chunk, (unsigned long long)p.src_node, got, p.crc);
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.verify_failures++;
  }
  set_chunk_ev(L, int64_t(c), 0);
  if (++L.fails[c] > cfg_.max_retries || !node_) {
    fail(std::string(buf) + (node_ ? " (retries exhausted)" : ""));
    return;
  }
  log::warn(int64_t(self_node_)).msg(std::string(buf) + "; requesting a re-send");
  trace::mark("dissem.crc_mismatch");
  L.st[c] = 4;
  if (p.kind == Kind::Local) {
    // The source bytes did not match their manifest on the way in: stage again
    // (after the poll loop; staging appends to verifies_).
    restage_.push_back({p.layer, p.chunk});
    return;
  }
  Message n;
  n.type = MsgType::Nack;
  n.layer = p.layer;
  n.dest = p.src_node;  // the sender whose bytes failed
  n.offset = p.off;
  n.data_size = p.len;
  n.total_size = p.total;
  node_->send_msg(node_->leader(), n);
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.nacks++;
}

void PlannedEngine::stage_chunk(Layer& L, LayerID id, int64_t c) {
  if (!L.host && L.path.empty()) {
    LayerSrc src;
    if (!node_ || !node_->store().get(id, &src) || (!src.host && src.path.empty()))
      throw std::runtime_error("layer " + std::to_string(id) + " has no host or disk source to stage");
    if (src.host) {
      L.host = src.host->ptr + src.offset;
    } else {
      L.path = src.path;
      L.path_off = src.offset;
    }
  }
  if (L.host) {
    stage_from(L, id, c, L.host + c * src_grid(L), nullptr);
  } else {
    submit_disk(L, id, c);
  }
}

void PlannedEngine::submit_disk(Layer& L, LayerID id, int64_t c) {
  if (readers_.empty()) {
    if (cfg_.node_disk_rate > 0 && !pacer_)
      pacer_ = std::make_unique<NodePacer>(cfg_.node_disk_key.empty() ? "default" : cfg_.node_disk_key,
                                           cfg_.node_disk_rate);
    for (int i = 0; i < std::max(1, cfg_.disk_ring); ++i) {
      uint8_t* b = backend_->alloc_host(cfg_.chunk_bytes);
      bounce_all_.push_back(b);
      bounce_free_.push_back(b);
    }
    for (int i = 0; i < std::max(1, cfg_.disk_readers); ++i) readers_.push_back(vclock::spawn([this] { reader_loop(); }, "disk-reader"));
  }
  L.st[size_t(c)] = 3;
  DiskRead d;
  d.layer = id;
  d.chunk = c;
  d.file_off = L.path_off + c * src_grid(L);
  d.len = src_len(L, c);
  d.path = L.path;
  disk_wait_.push_back(std::move(d));
  pump_disk();
}

void PlannedEngine::pump_disk() {
  // Buffers whose H2D copy landed go back to the ring.
  for (auto it = bounce_busy_.begin(); it != bounce_busy_.end();) {
    const int r = backend_->query(it->first);
    if (r == 0) {
      ++it;
      continue;
    }
    ev_drop(it->first);
    bounce_free_.push_back(it->second);
    it = bounce_busy_.erase(it);
  }
  // Hand waiting reads to the readers while bounce buffers are free.
  while (!disk_wait_.empty() && !bounce_free_.empty()) {
    DiskRead d = std::move(disk_wait_.front());
    disk_wait_.pop_front();
    d.bounce = bounce_free_.back();
    bounce_free_.pop_back();
    disk_inflight_++;
    {
      std::lock_guard<std::mutex> lk(disk_mu_);
      disk_todo_.push_back(std::move(d));
    }
    disk_cv_.notify_one();
  }
  // Reads that finished: DMA them into HBM from their bounce buffer.
  std::deque<DiskRead> done;
  {
    std::lock_guard<std::mutex> lk(disk_mu_);
    done.swap(disk_done_);
  }
  for (auto& d : done) {
    disk_inflight_--;
    if (!d.ok) {
      fail("disk read failed for layer " + std::to_string(d.layer) + " chunk " + std::to_string(d.chunk));
      continue;
    }
    Layer& L = layers_[d.layer];
    stage_from(L, d.layer, d.chunk, d.bounce, d.bounce);
  }
}

void PlannedEngine::reader_loop() {
  std::map<std::string, int> fds;
  std::map<std::string, bool> direct;  // path -> opened with O_DIRECT
  for (;;) {
    DiskRead d;
    {
      std::unique_lock<std::mutex> lk(disk_mu_);
      disk_cv_.wait(lk, [&] { return !disk_todo_.empty() || stop_req_.load(); });
      if (disk_todo_.empty()) break;
      d = std::move(disk_todo_.front());
      disk_todo_.pop_front();
    }
    int& fd = fds[d.path];
    if (fd <= 0) {
      fd = cfg_.disk_o_direct ? ::open(d.path.c_str(), O_RDONLY | O_DIRECT | O_CLOEXEC) : -1;
      direct[d.path] = fd >= 0;
      if (fd < 0) {
        // e.g. an old tmpfs: no O_DIRECT. Still read, but say so: these bytes
        // may come from the page cache, and the stats count them apart
        // (disk_buffered_bytes; bench.py refuses such a run without --allow-buffered).
        fd = ::open(d.path.c_str(), O_RDONLY | O_CLOEXEC);
        if (cfg_.disk_o_direct)
          log::warn(int64_t(self_node_)).s("path", d.path).msg("O_DIRECT refused: buffered disk reads");
      }
    }
    // O_DIRECT needs 4 KiB aligned lengths; the bounce buffer holds a whole chunk.
    const int64_t want = std::min<int64_t>(((d.len + 4095) / 4096) * 4096, cfg_.chunk_bytes);
    if (pacer_) {  // the node's one NVMe: wait for this read's slot in the shared budget
      const int64_t w = pacer_->acquire(want);
      std::lock_guard<std::mutex> lk(stats_mu_);
      stats_.disk_wait_ms += double(w) / 1e6;
    }
    int64_t got = 0;
    while (fd >= 0 && got < d.len) {
      ssize_t r = ::pread(fd, d.bounce + got, size_t(want - got), off_t(d.file_off + got));
      if (r <= 0) break;
      got += r;
    }
    d.ok = got >= d.len;
    {
      std::lock_guard<std::mutex> lk(stats_mu_);
      (direct[d.path] ? stats_.disk_direct_bytes : stats_.disk_buffered_bytes) += got;
    }
    {
      std::lock_guard<std::mutex> lk(disk_mu_);
      disk_done_.push_back(std::move(d));
    }
    req_cv_.notify_all();
  }
  for (auto& kv : fds)
    if (kv.second > 0) ::close(kv.second);
}

void PlannedEngine::stage_from(Layer& L, LayerID id, int64_t c, const uint8_t* src, uint8_t* bounce) {
  const int64_t off = c * grid_;
  const int64_t len = std::min(grid_, L.size - off);
  const int64_t slen = src_len(L, c);
  trace::Scoped tr("dissem.stage");
  if (!L.dev) L.dev = backend_->alloc(L.size);
  Ev e = cfg_.pack == 1 && !L.src_packed ? backend_->stage_pack(L.dev + off, src, slen, cfg_.pack_block)
                                         : backend_->stage(L.dev + off, src, len);
  L.st[size_t(c)] = 1;
  L.rkey[size_t(c)] = Key{};
  set_chunk_ev(L, c, e);
  Piece p{Kind::Local, 0, 0, cfg_.rank, id, off, len, L.size, c, true};
  p.src_node = self_node_;
  // The chunk's expected CRC: this rank's manifest of the layer, or - for a
  // layer it stages from a node-shared host copy it did not generate - the
  // CRC the leader put in the job.
  uint32_t want = 0;
  bool known = false;
  if (int64_t(L.manifest.crc.size()) > c) {
    want = L.manifest.crc[size_t(c)];
    known = true;
  } else if (auto jc = L.job_crc.find(c); jc != L.job_crc.end()) {
    want = jc->second;
    known = true;
  }
  // The check joins the pending batch (flush_checks): one verify launch per
  // kVerifyBatch staged chunks instead of one per chunk.
  PendingCheck sc;
  sc.wait = e;
  sc.held = true;
  ev_hold(e);
  if (cfg_.unpack_store) {
    // fused: check the packed chunk and write its bf16 image (one pass)
    const bool check = cfg_.verify && known;
    if (check) {
      p.has_crc = true;
      p.crc = want;
    }
    const uint32_t slot = crc_slot();
    sc.req = unpack_req(L, c, slot);
    sc.has_req = true;
    sc.slot = check ? slot : ~0u;
  } else if (cfg_.verify && known) {
    p.has_crc = true;
    p.crc = want;
    sc.slot = crc_slot();
    sc.req = Backend::CheckReq{L.dev + off, len, sc.slot};
    sc.has_req = true;
  }
  sc.piece = p;
  pending_checks_.push_back(sc);
  pending_reqs_ += sc.has_req ? 1 : 0;  // checks to launch, as issue_lane counts them
  if (pending_reqs_ >= kVerifyBatch) flush_checks();
  if (bounce) {
    // The bounce buffer is free again once its H2D copy has landed - not after
    // the chunk's CRC check: the verify queue is in order, and a check queued
    // behind a recv that waits on a peer (whose send may wait on a disk read of
    // its own) would hold every buffer of the ring - two ranks deadlock.
    ev_hold(e);
    bounce_busy_.push_back({e, bounce});
  }
  std::lock_guard<std::mutex> lk(stats_mu_);
  stats_.bytes_staged += slen;
}

// The checks queued since the last flush (staged chunks, and the chunks the
// P2P groups of this issue pass landed) go to the verify queue as batches of
// up to kVerifyBatch chunk checks, each batch one Backend::verify behind the
// landings of its own chunks only, so verification keeps pipelining behind
// staging and transfers.
void PlannedEngine::flush_checks() {
  size_t i = 0;
  while (i < pending_checks_.size()) {
    Verify v;
    v.t0 = pending_checks_[i].t0;
    std::vector<Backend::CheckReq> reqs;
    std::vector<Ev> waits;
    size_t j = i;
    for (; j < pending_checks_.size(); ++j) {
      const PendingCheck& pc = pending_checks_[j];
      if (pc.has_req && reqs.size() == size_t(kVerifyBatch)) break;
      if (pc.has_req) {
        reqs.push_back(pc.req);
        reqs.back().expect = pc.piece.has_crc ? pc.piece.crc : 0;
      }
      if (pc.wait && std::find(waits.begin(), waits.end(), pc.wait) == waits.end()) waits.push_back(pc.wait);
      v.pieces.push_back(pc.piece);
      v.slots.push_back(pc.slot);
    }
    v.ev = backend_->verify(reqs, waits);
    verifies_.push_back(std::move(v));
    i = j;
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.verify_calls++;
    stats_.verify_chunks += int64_t(reqs.size());
  }
  drop_pending_checks();
}

void PlannedEngine::drop_pending_checks() {
  for (auto& pc : pending_checks_)
    if (pc.held) ev_drop(pc.wait);
  pending_checks_.clear();
  pending_reqs_ = 0;
  for (Ev e : owned_waits_) backend_->release(e);
  owned_waits_.clear();
}

int PlannedEngine::ensure_chunk(Layer& L, LayerID id, int64_t c, bool want_landed) {
  if (want_landed) L.want[size_t(c)] = 1;
  uint8_t s = L.st[size_t(c)];
  if (s == 2) {
    if (want_landed) {
      const int64_t off = c * grid_;
      Piece p{Kind::Local, 0, 0, cfg_.rank, id, off, std::min(grid_, L.size - off), L.size, c, true};
      p.src_node = self_node_;
      landed(p);
      L.want[size_t(c)] = 0;
    }
    return 1;
  }
  if (s == 1) return 1;
  if (s == 3) return 0;  // disk read in flight
  if (s == 4 && !want_landed) return 1;  // forward the bad copy; its receiver NACKs it as well
  if (L.host && L.host_prefix >= 0) {
    // A client stream still landing in host memory: its chunks stage as they
    // complete (cut-through); a later one waits for host_prefix_ready.
    if (c * src_grid(L) + src_len(L, c) > L.host_prefix) return 0;
    if (s == 0 && stage_paced(L, id, c)) {
      if (want_landed) local_wait_.push_back({id, c});
      return 0;
    }
    stage_chunk(L, id, c);
    return L.st[size_t(c)] == 1 ? 1 : 0;
  }
  LayerSrc src;
  const bool have = node_ && node_->store().get(id, &src);
  // A client layer's host buffer exists while its stream is still landing; it
  // becomes a source only once the node re-tags it Inmem (Node::on_layer).
  const bool client = have && src.meta.location == Location::Client;
  if (L.host || !L.path.empty() || (have && !client && (src.host || !src.path.empty()))) {
    if (!source_covers(L, id, c)) {
      // A hole of a resumed partial copy: a send of it waits for the chunk's
      // recv; a promotion of it has no source here.
      return want_landed ? -1 : 0;
    }
    if (s == 0 && stage_paced(L, id, c)) {
      // The source tier's LimitRate holds this chunk back; promotions retry from
      // local_wait_, sends from their lane's next issue pass.
      if (want_landed) local_wait_.push_back({id, c});
      return 0;
    }
    stage_chunk(L, id, c);
    return L.st[size_t(c)] == 1 ? 1 : 0;
  }
  if (client) {
    // Held by this node's external client (client.go): ask for the layer once.
    // It arrives over TCP into host memory; the node then calls load_range,
    // and this chunk (and any send waiting on it) stages from that copy.
    if (!L.client_requested) {
      L.client_requested = true;
      node_->request_client_layer(id);
    }
    return 0;
  }
  return -1;
}

bool PlannedEngine::has_local_source(Layer& L, LayerID id, int64_t c) {
  if (!source_covers(L, id, c)) return false;
  if (L.host || !L.path.empty()) return true;
  LayerSrc src;
  return node_ && node_->store().get(id, &src) &&
         (src.host || !src.path.empty() || src.meta.location == Location::Client);
}

bool PlannedEngine::source_covers(Layer& L, LayerID id, int64_t c) {
  // A resumed partial copy (LayerSrc::ranges) holds only some chunks; the
  // others are holes of its sparse file and must arrive over the wire first.
  if (!L.ranges_known) {
    LayerSrc src;
    L.src_ranges.clear();
    if (node_ && node_->store().get(id, &src)) L.src_ranges = src.ranges;
    L.ranges_known = true;
  }
  if (L.src_ranges.empty()) return true;
  const int64_t a = c * grid_, b = std::min(a + grid_, L.size);
  for (auto& r : L.src_ranges)
    if (r.first <= a && r.second >= b) return true;
  return false;
}

}  // namespace dissem
