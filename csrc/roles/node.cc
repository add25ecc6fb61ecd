#include "roles/node.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <set>
#include <tuple>

#include "core/log.h"
#include "core/trace.h"
#include "sched/maxflow.h"

namespace dissem {

namespace {
bool at(const LayerIDs& ids, LayerID l, Location loc) {
  auto it = ids.find(l);
  return it != ids.end() && it->second.location == loc;
}
}  // namespace

Node::Node(NodeConfig cfg, std::shared_ptr<Transport> t, std::shared_ptr<DataEngine> e, const LayersSrc& layers,
           const Assignment& assignment, bool is_leader)
    : cfg_(std::move(cfg)),
      t_(std::move(t)),
      e_(std::move(e)),
      store_(layers, e_->target()),
      assignment_(assignment),
      is_leader_(is_leader),
      rng_(cfg_.seed) {
  if (cfg_.id != cfg_.leader) add_node(cfg_.leader);  // node.go:58-60
  if (is_leader_) {
    status_[cfg_.id] = store_.inventory();  // node.go:252-257
    partial_[cfg_.id] = store_.partial();
    for (auto& kv : cfg_.link_report) measured_links_[{cfg_.id, kv.first}] = kv.second;
  }
  e_->bind(this);
  if (is_leader_ && e_->planned()) {
    // Whole copies only, the filter announce() applies: a resumed partial copy's
    // manifest holds CRC 0 for every chunk it lacks. Its real chunks are merged
    // per chunk (merge_partial_manifest), like any other partial holder's.
    const LayerIDs inv = store_.inventory();
    const PartialLayers part = store_.partial();
    for (auto& kv : e_->manifest()) {
      if (inv.count(kv.first)) manifests_[kv.first] = kv.second;
      auto pit = part.find(kv.first);
      if (pit != part.end()) merge_partial_manifest(kv.first, kv.second, pit->second);
    }
  }
  // TCP payload bytes land directly in this node's host slot of the layer
  // (host engines: the target itself; GPU engines: the staging source of a
  // client-held layer, see on_layer).
  LandingFn landing = [this](const Message& h) -> uint8_t* {
    if (h.epoch && cfg_.epoch && h.epoch != cfg_.epoch) return nullptr;
    try {
      int64_t total = h.total_size ? h.total_size : h.data_size;
      if (h.offset < 0 || h.offset + h.data_size > total) return nullptr;
      return store_.host_landing(h.layer, total) + h.offset;
    } catch (...) {
      return nullptr;
    }
  };
  ProgressFn progress;
  if (e_->target() == Location::Device) {
    // Cut-through (transport.go:144-196, at chunk grain): while a client
    // stream is still arriving, every chunk that has fully landed in host
    // memory is handed to the engine, which stages it into HBM and forwards it
    // to the dests waiting on it before the rest of the layer is here.
    progress = [this](const Message& h, int64_t got) {
      if (h.epoch && cfg_.epoch && h.epoch != cfg_.epoch) return;
      if (h.offset != 0) return;  // client streams carry whole layers from offset 0
      const int64_t total = h.total_size ? h.total_size : h.data_size;
      const int64_t step = std::max<int64_t>(e_->chunk_bytes(), 1);
      const int64_t prefix = got >= total ? total : (got / step) * step;
      {
        std::lock_guard<std::mutex> lk(stream_mu_);
        int64_t& done = stream_prefix_[h.layer];
        if (prefix <= done) return;
        done = prefix;
      }
      e_->host_prefix_ready(h.layer, store_.host_landing(h.layer, total), prefix, total);
    };
  }
  t_->set_hooks(this, std::move(landing), std::move(progress));
}

Node::~Node() {
  stop();
  t_->clear_hooks(this);
}

void Node::start() {
  if (running_.exchange(true)) return;
  loop_th_ = std::thread([this] { loop(); });
  if (is_leader_) {
    // A leader whose assignment names only itself gets no announce: check once at start.
    auto m = std::make_shared<Message>();
    m->type = MsgType::Tick;
    m->epoch = cfg_.epoch;
    t_->inject(m);
    if (cfg_.job_timeout_s > 0) tick_th_ = std::thread([this] { ticker(); });
  }
}

void Node::ticker() {
  // Deadline checks run on the event loop: this thread only posts Ticks.
  const double period = std::min(0.25, std::max(0.01, cfg_.job_timeout_s / 4));
  std::unique_lock<std::mutex> lk(tick_mu_);
  while (!cv_wait_for(tick_cv_, lk, period, [&] { return tick_stop_; })) {
    auto m = std::make_shared<Message>();
    m->type = MsgType::Tick;
    m->epoch = cfg_.epoch;
    t_->inject(m);
  }
}

void Node::stop() {
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> lk(tick_mu_);
    tick_stop_ = true;
  }
  tick_cv_.notify_all();
  if (tick_th_.joinable()) tick_th_.join();
  e_->quiesce();
  auto m = std::make_shared<Message>();
  m->type = MsgType::Stop;
  t_->inject(m);
  if (loop_th_.joinable()) loop_th_.join();
}

void Node::add_routing(NodeID goal, NodeID next_hop, unsigned hops) {
  std::lock_guard<std::mutex> lk(rt_mu_);
  routing_[goal] = {next_hop, hops};
}

NodeID Node::next_hop(NodeID goal) {
  std::lock_guard<std::mutex> lk(rt_mu_);
  auto it = routing_.find(goal);
  if (it == routing_.end()) throw std::runtime_error("routing entry for the specified the goal does not exist");
  return it->second.first;
}

std::map<std::pair<NodeID, NodeID>, int64_t> Node::plan_link_bw() {
  std::lock_guard<std::mutex> lk(sig_mu_);
  return cfg_.link_bw;
}

void Node::update_leader(NodeID leader) {
  std::lock_guard<std::mutex> lk(rt_mu_);
  if (!routing_.count(leader)) throw std::runtime_error("routing entry for the specified leader does not exist");
  cfg_.leader = leader;
}

bool Node::send_msg(NodeID dest, Message m) {
  m.src = cfg_.id;
  m.epoch = cfg_.epoch;
  try {
    t_->send(dest, m);
    return true;
  } catch (const std::exception& e) {
    log::error(int64_t(cfg_.id)).s("error", e.what()).msg(std::string("failed to send ") + msg_type_name(m.type) +
                                                          " to " + std::to_string(dest));
    return false;
  }
}

void Node::announce() {
  if (is_leader_ && cfg_.id == cfg_.leader) return;  // the leader's status is seeded at construction
  Message m;
  m.type = MsgType::Announce;
  m.layers = store_.inventory();
  m.partial_layers = store_.partial();
  m.link_rates = cfg_.link_report;
  if (e_->planned()) {
    // Whole copies' manifests, and a resumed partial copy's too: the leader
    // takes from the latter only the chunks inside its announced ranges.
    for (auto& kv : e_->manifest())
      if (m.layers.count(kv.first) || m.partial_layers.count(kv.first)) m.manifest[kv.first] = kv.second;
  }
  NodeID hop = next_hop(cfg_.leader);
  trace::mark("dissem.announce");
  if (!send_msg(hop, m)) throw std::runtime_error("announce failed");
}

bool Node::wait_ready(double timeout_s) {
  std::unique_lock<std::mutex> lk(sig_mu_);
  return cv_wait_for(sig_cv_, lk, timeout_s, [&] { return is_leader_ ? satisfied_ : ready_; });
}

bool Node::wait_start(double timeout_s) {
  std::unique_lock<std::mutex> lk(sig_mu_);
  return cv_wait_for(sig_cv_, lk, timeout_s, [&] { return started_; });
}

Status Node::status() {
  // Snapshot through the event loop would be cleaner; status_ is only written on the
  // loop thread and this accessor is for tests after completion.
  std::lock_guard<std::mutex> lk(sig_mu_);
  return status_;
}

NodeStats Node::stats() {
  std::lock_guard<std::mutex> lk(sig_mu_);
  return stats_;
}

void Node::loop() {
  for (;;) {
    auto m = t_->deliver().pop();
    if (!m) break;
    if ((*m)->type == MsgType::Stop) break;
    try {
      handle(*m);
    } catch (const std::exception& e) {
      log::error(int64_t(cfg_.id)).s("error", e.what()).msg(std::string("handler failed for ") +
                                                          msg_type_name((*m)->type));
    }
  }
}

void Node::handle(const MessagePtr& m) {
  if (m->epoch && cfg_.epoch && m->epoch != cfg_.epoch) {
    log::debug(int64_t(cfg_.id)).u("epoch", m->epoch).msg("dropping message from another session");
    return;
  }
  if (log::level() <= log::Debug)
    log::debug(int64_t(cfg_.id)).msg(std::string("incoming msg[") + msg_type_name(m->type) + "]: " + m->str());
  if (e_->on_message(m)) return;
  switch (m->type) {
    case MsgType::Announce:
      if (is_leader_) on_announce(m);
      break;
    case MsgType::Ack:
      if (is_leader_) m->partial ? on_range_ack(m) : on_ack(m);
      break;
    case MsgType::Layer:
      on_layer(m);
      break;
    case MsgType::Landed:
      on_landed(m->layer, m->offset, m->data_size, m->total_size, m->src, m->dur_ms);
      break;
    case MsgType::Retransmit:
      on_retransmit(m);
      break;
    case MsgType::FlowRetransmit:
      on_flow_retransmit(m);
      break;
    case MsgType::Startup:
      on_startup(m);
      break;
    case MsgType::Simple:
      log::info(int64_t(cfg_.id)).s("from", m->src_addr).msg(m->payload_str);
      break;
    case MsgType::Nack:
      if (is_leader_) on_nack(m);
      break;
    case MsgType::Suspect:
      if (is_leader_) on_suspect(m);
      break;
    case MsgType::ShrinkDone:
      // From this node's engine (via the inbox, behind its earlier acks).
      if (is_leader_) on_shrink_done(m);
      else send_msg(cfg_.leader, *m);
      break;
    case MsgType::Tick:
      if (is_leader_ && !started_) {
        bool all = true;
        for (auto& kv : assignment_) all = all && status_.count(kv.first);
        if (all && !assignment_.empty()) start_distribution();
      } else if (is_leader_) {
        on_tick();
      }
      break;
    default:
      break;
  }
}

// ------------------------------------------------------------ receiver side

void Node::on_layer(const MessagePtr& m) {
  // A payload that arrived over the transport (node.go:1354-1384 / 1520-1567).
  int64_t total = m->total_size ? m->total_size : m->data_size;
  if (e_->target() == Location::Device && (m->in_place || m->data)) {
    // Device target: the host copy (e.g. from the external client) is the
    // staging source; the engine reports Landed once the bytes are in HBM.
    // Chunks that landed while the stream was arriving are already staged
    // (set_progress above); this stages whatever is left.
    uint8_t* dst = store_.host_landing(m->layer, total);
    if (!m->in_place) memcpy(dst + m->offset, m->data->ptr + m->data_off, size_t(m->data_size));
    LayerSrc src;
    if (store_.get(m->layer, &src)) {
      src.meta.location = Location::Inmem;
      store_.put(m->layer, src);
    }
    if (m->offset == 0 && m->data_size == total) e_->host_prefix_ready(m->layer, dst, total, total);
    e_->load_range(m->layer, m->offset, m->data_size, total, 0);
    return;
  }
  if (!m->in_place && m->data) {
    uint8_t* dst = store_.host_landing(m->layer, total);
    if (m->offset < 0 || m->offset + m->data_size > total) throw std::runtime_error("layer range out of bounds");
    memcpy(dst + m->offset, m->data->ptr + m->data_off, size_t(m->data_size));
  }
  on_landed(m->layer, m->offset, m->data_size, total, m->src, m->dur_ms);
}

void Node::on_landed(LayerID layer, int64_t off, int64_t size, int64_t total, NodeID from, double dur_ms) {
  bool complete = store_.mark_landed(layer, off, size, total);
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.bytes_received += size;
  }
  if (size < total && !complete) {
    log::info(int64_t(cfg_.id)).msg("l" + std::to_string(layer) + " downloaded (" +
                                    std::to_string(store_.landed_bytes(layer)) + " B / " + std::to_string(total) +
                                    " B)");
    if (cfg_.range_acks && cfg_.id != kClientID) {  // mode-2 range jobs retire on these
      Message a;
      a.type = MsgType::Ack;
      a.layer = layer;
      a.location = e_->target();
      a.partial = true;
      a.offset = off;
      a.data_size = size;
      send_msg(cfg_.leader, a);
    }
  }
  if (complete) {
    log::info(int64_t(cfg_.id)).u("layer", layer).i("total_bytes", total).u("from", from).f("duration[ms]", dur_ms)
        .msg("layer fully received");
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.layers_received++;
    }
    send_ack(layer);
  }
}

void Node::send_ack(LayerID layer) {
  Message a;
  a.type = MsgType::Ack;
  a.layer = layer;
  a.location = e_->target();
  send_msg(cfg_.leader, a);
}

void Node::on_retransmit(const MessagePtr& m) {
  // node.go:1462-1484: add the dest as a neighbor, then push our copy.
  add_node(m->dest);
  LayerSrc src;
  if (!store_.get(m->layer, &src)) {
    log::warn(int64_t(cfg_.id)).msg("no layers found for layerID:" + std::to_string(m->layer));
    return;
  }
  send_layer(m->dest, m->layer, 0, src.data_size, src.meta.limit_rate);
}

void Node::on_flow_retransmit(const MessagePtr& m) {
  // node.go:1592-1643 (sender side of mode 3, also self-loads when dest == me).
  add_node(m->dest);
  log::info(int64_t(cfg_.id)).u("layer", m->layer).u("dest", m->dest).i("size", m->data_size).i("rate", m->rate)
      .msg("start sending layer");
  send_layer(m->dest, m->layer, m->offset, m->data_size, m->rate);
}

void Node::on_startup(const MessagePtr&) {
  // node.go:1387-1389: tell the application the layers are ready.
  trace::mark("dissem.startup");
  std::lock_guard<std::mutex> lk(sig_mu_);
  ready_ = true;
  sig_cv_.notify_all();
}

// -------------------------------------------------------------- sender side

void Node::send_layer(NodeID dest, LayerID layer, int64_t offset, int64_t size, int64_t rate) {
  LayerSrc src;
  if (!store_.get(layer, &src)) {
    log::warn(int64_t(cfg_.id)).msg("no layers found for layerID:" + std::to_string(layer));
    return;
  }
  int64_t total = src.data_size;
  if (size < 0 || offset + size > total) size = total - offset;
  if (dest == cfg_.id) {
    // Local promotion into the target tier (the reference sends to itself over
    // TCP loopback, node.go:1239-1247 / mode-2 own jobs).
    if (store_.has_target(layer)) {
      send_ack(layer);  // already resident: acks are idempotent at the leader
      return;
    }
    if (src.meta.location == Location::Client) {
      fetch_from_client(layer, cfg_.id);
      return;
    }
    e_->load_range(layer, offset, size, total, rate);
    return;
  }
  if (src.meta.location == Location::Client && !store_.has_target(layer)) {
    fetch_from_client(layer, dest);  // node.go:357-361 / 1470-1474
    return;
  }
  e_->send_range(dest, layer, offset, size, total, rate);
}

void Node::request_client_layer(LayerID layer) {
  log::info(int64_t(cfg_.id)).u("layerID", layer).msg("ask the client to send the layer (device staging)");
  Message r;
  r.type = MsgType::ClientReq;
  r.layer = layer;
  send_msg(kClientID, r);
}

void Node::fetch_from_client(LayerID layer, NodeID dest) {
  log::debug(int64_t(cfg_.id)).u("layerID", layer).msg("ask the client to send the layer");
  if (dest != cfg_.id) {
    try {
      t_->register_pipe(layer, dest);
    } catch (const std::exception& e) {
      log::error(int64_t(cfg_.id)).s("error", e.what()).msg("register pipe");
    }
  }
  Message r;
  r.type = MsgType::ClientReq;
  r.layer = layer;
  r.save_disk = false;
  send_msg(kClientID, r);
}

// -------------------------------------------------------------- leader side

int64_t Node::layer_size(LayerID l) {
  int64_t sz = 0;
  for (auto& kv : status_) {
    auto it = kv.second.find(l);
    if (it != kv.second.end()) sz = std::max(sz, it->second.size);
  }
  if (!sz) {
    LayerSrc src;
    if (store_.get(l, &src)) sz = src.data_size;
  }
  return sz;
}

void Node::on_announce(const MessagePtr& m) {
  // node.go:295-324
  if (!status_.count(m->src)) {
    std::lock_guard<std::mutex> lk(sig_mu_);
    status_[m->src] = m->layers;
    partial_[m->src] = m->partial_layers;
    add_node(m->src);
    for (auto& kv : m->link_rates) measured_links_[{m->src, kv.first}] = kv.second;
  }
  for (auto& kv : m->manifest) {
    auto pit = m->partial_layers.find(kv.first);
    if (pit != m->partial_layers.end()) {  // a partial copy vouches for its own chunks only
      merge_partial_manifest(kv.first, kv.second, pit->second);
      continue;
    }
    auto it = manifests_.find(kv.first);
    if (it == manifests_.end()) {
      manifests_[kv.first] = kv.second;
    } else if (it->second.chunk_bytes == kv.second.chunk_bytes && it->second.crc != kv.second.crc) {
      log::error(int64_t(cfg_.id)).u("layer", kv.first).u("from", m->src).msg("conflicting CRC manifest for layer");
    }
  }
  if (started_) return;
  for (auto& kv : assignment_)
    if (!status_.count(kv.first)) return;
  start_distribution();
}

void Node::start_distribution() {
  int64_t planned = 0;
  for (auto& kv : assignment_)
    for (auto& l : kv.second)
      if (!at(status_[kv.first], l.first, e_->target())) planned += layer_size(l.first);
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    started_ = true;
    t_start_us_ = log::now_us();
    stats_.bytes_planned = planned;
    sig_cv_.notify_all();
  }
  initial_status_ = status_;
  if (cfg_.adapt_links && !measured_links_.empty()) {
    // Closed loop: plan on the rates the senders measured (reported with their
    // announces) instead of the estimates; links nobody measured keep theirs.
    std::lock_guard<std::mutex> lk(sig_mu_);
    for (auto& kv : measured_links_)
      if (kv.second > 0) cfg_.link_bw[kv.first] = kv.second;
  }
  log::info(int64_t(cfg_.id)).i("mode", cfg_.mode).i("bytes_planned", planned)
      .i("measured_links", int64_t(measured_links_.size())).msg("timer start");
  session_range_ = trace::start("dissem.session");
  int64_t t0 = log::now_us();
  {
    trace::Scoped plan("dissem.plan");
    switch (cfg_.mode) {
      case 0: schedule_mode0(); break;
      case 1: schedule_mode1(); break;
      case 2: schedule_mode2(); break;
      case 3: schedule_mode3(); break;
      default: log::error(int64_t(cfg_.id)).msg("unknown mode");
    }
    flush_batch();
  }
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.plan_ms = double(log::now_us() - t0) / 1e3;
  }
  if (!satisfied_ && assignment_satisfied()) {
    // Nothing had to move (the reference would wait forever for acks).
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      satisfied_ = true;
      t_ready_us_ = log::now_us();
      stats_.time_to_deliver_s = double(t_ready_us_ - t_start_us_) / 1e6;
    }
    log::info(int64_t(cfg_.id)).msg("timer stop: startup");
    trace::stop(session_range_);
    send_startup();
    std::lock_guard<std::mutex> lk(sig_mu_);
    sig_cv_.notify_all();
  }
}

bool Node::assignment_satisfied() {
  // node.go:435-446: every assigned layer must be resident in the target tier.
  for (auto& kv : assignment_) {
    auto st = status_.find(kv.first);
    if (st == status_.end()) return false;
    for (auto& l : kv.second)
      if (!at(st->second, l.first, e_->target())) return false;
  }
  return true;
}

void Node::send_startup() {
  // node.go:456-469 (continues past per-peer errors instead of returning early).
  for (auto& kv : status_) {
    Message s;
    s.type = MsgType::Startup;
    send_msg(kv.first, s);
  }
}

void Node::on_ack(const MessagePtr& m) {
  if (dead_nodes_.count(m->src)) return;  // sent before it died: it is out of the assignment
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    LayerMeta meta;
    meta.location = m->location;
    meta.size = layer_size(m->layer);
    status_[m->src][m->layer] = meta;  // node.go:413-417
  }
  outstanding_.erase({m->src, m->layer});
  finish_if_satisfied();
  if (cfg_.mode != 2) return;
  // Mode 2 pull loop (node.go:764-807): the whole layer is at the dest, so every
  // job of (layer, dest) is done; retire them and pull the next ones.
  auto lj = jobs_.find(m->layer);
  if (lj != jobs_.end()) {
    std::vector<JobKey> done;
    for (auto& kv : lj->second)
      if (kv.first.first == m->src) done.push_back(kv.first);
    for (auto& k : done) retire_job(m->layer, k);
  }
  // The destination now owns a copy it can serve (status grew above): let it pull too.
  while (inflight_[m->src] < cfg_.pull_window && assign_new_job(m->src)) {
  }
  flush_batch();
}

void Node::finish_if_satisfied() {
  if (satisfied_ || !assignment_satisfied()) return;
  // Fire exactly once (quirk Q13).
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    satisfied_ = true;
    t_ready_us_ = log::now_us();
    stats_.time_to_deliver_s = double(t_ready_us_ - t_start_us_) / 1e6;
  }
  log::info(int64_t(cfg_.id)).f("time_to_deliver_s", stats_.time_to_deliver_s).msg("timer stop: startup");
  trace::stop(session_range_);
  send_startup();
  std::lock_guard<std::mutex> lk(sig_mu_);
  sig_cv_.notify_all();
}

// ------------------------------------------- elastic recovery (planned data plane)
//
// The reference only sketches this (Leader interface TODOs `update(a)` and
// `crash(n node)`, distributor/node.go:215-219; a dead sender hangs the run,
// SURVEY §5.3).
// A rank whose P2P group stalls or fails reports the group's peers (Suspect).
// The leader probes them over the control plane; for peers that are gone it
// starts a recovery generation: the dead nodes leave the status and the
// assignment, every survivor shrinks the RCCL communicator around them
// (ncclCommShrink with NCCL_SHRINK_ABORT: in-flight groups are aborted) and
// resets what was in flight, and once all survivors have confirmed
// (ShrinkDone) the leader re-plans every unacked (dest, layer) from a live
// holder. Pairs without a live holder are dropped (logged, counted).
void Node::on_suspect(const MessagePtr& m) {
  if (!started_ || satisfied_) return;
  std::vector<NodeID> gone;
  for (NodeID p : m->peers) {
    if (p == cfg_.id || dead_nodes_.count(p) || !status_.count(p)) continue;
    if (!t_->alive(p)) gone.push_back(p);
  }
  if (gone.empty()) {
    log::info(int64_t(cfg_.id)).u("from", m->src).i("peers", int64_t(m->peers.size()))
        .msg("suspect report: every named peer answers; waiting");
    return;
  }
  shrink_gen_++;
  for (NodeID d : gone) dead_nodes_.insert(d);
  int64_t dropped = 0;
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    for (NodeID d : gone) {
      status_.erase(d);
      auto a = assignment_.find(d);
      if (a != assignment_.end()) {
        dropped += int64_t(a->second.size());
        assignment_.erase(a);
      }
    }
    stats_.recoveries++;
    stats_.dropped += dropped;
  }
  for (NodeID d : gone) initial_status_.erase(d);
  // Planning state of the interrupted schedule: re-planned from scratch.
  pending_jobs_.clear();
  jobs_.clear();
  load_.clear();
  inflight_.clear();
  outstanding_.clear();
  shrink_wait_.clear();
  for (auto& kv : status_) shrink_wait_.insert(kv.first);
  log::warn(int64_t(cfg_.id)).u("generation", shrink_gen_).i("dead", int64_t(gone.size()))
      .i("survivors", int64_t(shrink_wait_.size())).i("dropped_assignments", dropped)
      .msg("rank(s) dead: shrinking the communicator and re-planning");
  trace::mark("dissem.recovery");
  Message s;
  s.type = MsgType::Shrink;
  s.seq = shrink_gen_;
  s.peers.assign(dead_nodes_.begin(), dead_nodes_.end());
  s.payload_str = e_->new_comm_id();  // the survivors' new communicator (RCCL unique id)
  for (NodeID n : std::set<NodeID>(shrink_wait_)) send_msg(n, s);
}

void Node::on_shrink_done(const MessagePtr& m) {
  if (m->seq != shrink_gen_ || !shrink_wait_.erase(m->src)) return;
  if (shrink_wait_.empty()) replan_after_shrink();
}

void Node::replan_after_shrink() {
  const Location target = e_->target();
  std::map<NodeID, int64_t> planned;  // bytes per sender in this re-plan (spread the load)
  std::vector<std::pair<NodeID, LayerID>> lost;
  int64_t jobs = 0;
  for (auto& kv : assignment_) {
    const NodeID dest = kv.first;
    for (auto& l : kv.second) {
      const LayerID layer = l.first;
      auto st = status_.find(dest);
      if (st != status_.end() && at(st->second, layer, target)) continue;
      if (st != status_.end() && st->second.count(layer)) {
        add_job(dest, dest, layer, 0, -1);  // its own copy in another tier: promote it
        ++jobs;
        continue;
      }
      NodeID best = kClientID;
      for (auto& o : status_) {
        if (o.first == dest || !o.second.count(layer)) continue;
        if (best == kClientID || planned[o.first] < planned[best]) best = o.first;
      }
      if (best == kClientID) {
        lost.push_back({dest, layer});
        continue;
      }
      planned[best] += layer_size(layer);
      add_job(best, dest, layer, 0, -1);
      ++jobs;
    }
  }
  for (auto& dl : lost) {
    log::error(int64_t(cfg_.id)).u("dest", dl.first).u("layer", dl.second)
        .msg("no live holder of the layer: dropping it from the assignment");
    std::lock_guard<std::mutex> lk(sig_mu_);
    assignment_[dl.first].erase(dl.second);
    stats_.dropped++;
  }
  log::info(int64_t(cfg_.id)).u("generation", shrink_gen_).i("jobs", jobs).msg("re-planned after recovery");
  flush_batch();
  finish_if_satisfied();
}

void Node::on_range_ack(const MessagePtr& m) {
  // A range of a layer landed at m->src: range jobs it completes are retired.
  if (cfg_.mode != 2) return;
  auto lj = jobs_.find(m->layer);
  if (lj == jobs_.end()) return;
  std::vector<JobKey> done;
  for (auto& kv : lj->second) {
    if (kv.first.first != m->src) continue;
    Job& j = kv.second;
    const int64_t a = std::max(kv.first.second, m->offset);
    const int64_t b = std::min(kv.first.second + j.size, m->offset + m->data_size);
    if (a < b) j.got.add(a, b);
    if (j.got.covered() >= j.size) done.push_back(kv.first);
  }
  for (auto& k : done) retire_job(m->layer, k);
  if (!done.empty()) flush_batch();
}

void Node::retire_job(LayerID layer, const JobKey& key) {
  auto lj = jobs_.find(layer);
  if (lj == jobs_.end()) return;
  auto jt = lj->second.find(key);
  if (jt == lj->second.end()) return;
  Job job = jt->second;
  lj->second.erase(jt);
  if (job.state == JobState::Sending) {
    double dur = double(log::now_us() - job.t_us);
    auto& pf = perf_[job.sender];
    pf.first = pf.second == 0 ? dur : 0.5 * pf.first + 0.5 * dur;  // EWMA (quirk Q9)
    pf.second++;
    inflight_[job.sender] = std::max(0, inflight_[job.sender] - 1);
    log::info(int64_t(cfg_.id)).u("node", job.sender).u("layerID", layer).i("offset", key.second)
        .f("duration[ms]", dur / 1e3).msg("job completed");
  } else {
    load_[job.sender] = std::max<int64_t>(0, load_[job.sender] - 1);
  }
  while (inflight_[job.sender] < cfg_.pull_window && assign_new_job(job.sender)) {
  }
}

// ------------------------------------------------------- failure handling

void Node::track(NodeID sender, NodeID dest, LayerID layer, int64_t off, int64_t size) {
  if (cfg_.job_timeout_s <= 0 || !is_leader_) return;
  outstanding_[{dest, layer}].push_back({sender, off, size, log::now_us()});
}

NodeID Node::alternative_owner(LayerID layer, NodeID dest, NodeID avoid) {
  // Any live holder of the layer (announced or acked since), the least busy first.
  std::map<NodeID, int> busy;
  for (auto& kv : outstanding_)
    for (auto& o : kv.second) busy[o.sender]++;
  NodeID best = kClientID;
  int best_busy = INT_MAX;
  for (auto& kv : status_) {
    NodeID n = kv.first;
    if (n == dest || n == avoid || suspects_.count(n) || !kv.second.count(layer)) continue;
    if (busy[n] < best_busy) {
      best = n;
      best_busy = busy[n];
    }
  }
  return best;
}

void Node::on_tick() {
  if (!started_ || satisfied_ || cfg_.job_timeout_s <= 0 || e_->planned()) return;
  const int64_t now = log::now_us();
  struct Expired {
    NodeID dest;
    LayerID layer;
    Outstanding o;
  };
  std::vector<Expired> expired;
  for (auto it = outstanding_.begin(); it != outstanding_.end();) {
    auto& v = it->second;
    for (auto o = v.begin(); o != v.end();) {
      double allow = cfg_.job_timeout_s + (cfg_.job_min_rate > 0 ? double(o->size) / cfg_.job_min_rate : 0.0);
      if (double(now - o->t_us) / 1e6 > allow) {
        expired.push_back({it->first.first, it->first.second, *o});
        o = v.erase(o);
      } else {
        ++o;
      }
    }
    it = v.empty() ? outstanding_.erase(it) : std::next(it);
  }
  for (auto& e : expired) {
    if (!suspects_.count(e.o.sender) && e.o.sender != cfg_.id && e.o.sender != e.dest) {
      suspects_.insert(e.o.sender);
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.suspects++;
    }
    int& n = redispatches_[{e.dest, e.layer, e.o.off}];
    NodeID alt = alternative_owner(e.layer, e.dest, e.o.sender);
    if (alt == kClientID || ++n > cfg_.max_redispatch) {
      log::error(int64_t(cfg_.id)).u("layer", e.layer).u("dest", e.dest).u("sender", e.o.sender)
          .msg(alt == kClientID ? "job deadline expired and no other owner holds the layer"
                                : "job deadline expired too often; giving up on this range");
      track(e.o.sender, e.dest, e.layer, e.o.off, e.o.size);  // keep watching the original sender
      continue;
    }
    log::warn(int64_t(cfg_.id)).u("layer", e.layer).u("dest", e.dest).u("sender", e.o.sender).u("new_sender", alt)
        .i("offset", e.o.off).i("size", e.o.size).msg("job deadline expired: re-dispatching from another owner");
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.redispatched++;
    }
    if (cfg_.mode == 2) {
      // Keep the pull scheduler's books: the job now belongs to `alt`.
      auto lj = jobs_.find(e.layer);
      if (lj != jobs_.end()) {
        auto jt = lj->second.find({e.dest, e.o.off});
        if (jt != lj->second.end()) {
          if (jt->second.state == JobState::Sending) inflight_[jt->second.sender] = std::max(0, inflight_[jt->second.sender] - 1);
          jt->second.sender = alt;
          jt->second.state = JobState::Sending;
          jt->second.t_us = now;
          inflight_[alt]++;
        }
      }
    }
    if (e.o.off == 0 && e.o.size >= layer_size(e.layer)) {
      retransmit(e.layer, alt, e.dest);
    } else {
      track(alt, e.dest, e.layer, e.o.off, e.o.size);
      if (alt == cfg_.id) {
        send_layer(e.dest, e.layer, e.o.off, e.o.size, 0);
      } else {
        Message f;
        f.type = MsgType::FlowRetransmit;
        f.layer = e.layer;
        f.dest = e.dest;
        f.offset = e.o.off;
        f.data_size = e.o.size;
        send_msg(alt, f);
      }
    }
  }
  if (cfg_.mode == 2 && !expired.empty()) {
    // Pending jobs queued on a suspect move to live senders.
    for (auto& lj : jobs_)
      for (auto& jd : lj.second)
        if (jd.second.state == JobState::Pending && suspects_.count(jd.second.sender)) {
          load_[jd.second.sender] = std::max<int64_t>(0, load_[jd.second.sender] - 1);
          NodeID s = min_loaded_sender(lj.first, jd.first.first);
          if (s == kClientID) continue;
          jd.second.sender = s;
          load_[s]++;
        }
    for (auto& kv : load_)
      if (!suspects_.count(kv.first))
        while (inflight_[kv.first] < cfg_.pull_window && assign_new_job(kv.first)) {
        }
  }
}

void Node::on_nack(const MessagePtr& m) {
  // A receiver's chunk failed its CRC (planned engines): re-send that range,
  // preferably from a holder that had the layer before the session started
  // (its copy was checked against the manifest when it was staged).
  const NodeID dest = m->src, bad = m->dest;
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.nacks++;
  }
  std::vector<NodeID> cand;
  for (auto& kv : initial_status_)
    if (kv.first != dest && kv.first != bad && kv.second.count(m->layer)) cand.push_back(kv.first);
  NodeID src = bad;
  if (!cand.empty()) src = cand[size_t(rng_() % cand.size())];
  log::warn(int64_t(cfg_.id)).u("layer", m->layer).u("dest", dest).u("bad_sender", bad).u("new_sender", src)
      .i("offset", m->offset).i("size", m->data_size).msg("chunk failed its CRC: re-sending");
  if (!e_->planned()) return;
  add_job(src, dest, m->layer, m->offset, m->data_size);
  flush_batch();
}

void Node::add_job(NodeID src, NodeID dst, LayerID layer, int64_t offset, int64_t size, int phase, int64_t rate) {
  XferJob j;
  j.rate = rate;
  j.src = src;
  j.dst = dst;
  j.layer = layer;
  j.total = layer_size(layer);
  j.offset = offset;
  j.size = size < 0 ? j.total - offset : size;
  auto it = manifests_.find(layer);
  j.chunk_bytes = e_->chunk_bytes();
  if (it != manifests_.end() && it->second.chunk_bytes > 0) {
    j.chunk_bytes = it->second.chunk_bytes;
    int64_t first = j.offset / j.chunk_bytes;
    int64_t last = (j.offset + j.size + j.chunk_bytes - 1) / j.chunk_bytes;
    for (int64_t c = first; c < last && c < int64_t(it->second.crc.size()); ++c) j.crc.push_back(it->second.crc[size_t(c)]);
  } else if (auto pc = partial_crc_.find(layer); pc != partial_crc_.end() && pc->second.first > 0) {
    // No whole copy announced a manifest: the chunks partial holders vouched
    // for. One unknown chunk leaves the job unverified (never a wrong CRC).
    j.chunk_bytes = pc->second.first;
    const int64_t first = j.offset / j.chunk_bytes, last = (j.offset + j.size + j.chunk_bytes - 1) / j.chunk_bytes;
    for (int64_t c = first; c < last; ++c) {
      auto ci = pc->second.second.find(c);
      if (ci == pc->second.second.end()) {
        j.crc.clear();
        break;
      }
      j.crc.push_back(ci->second);
    }
  }
  pending_jobs_.push_back({j, phase});
}

void Node::merge_partial_manifest(LayerID layer, const CrcManifest& m,
                                  const std::vector<std::pair<int64_t, int64_t>>& ranges) {
  if (m.chunk_bytes <= 0) return;
  auto& pc = partial_crc_[layer];
  if (pc.first && pc.first != m.chunk_bytes) return;  // another grid: keep the first
  pc.first = m.chunk_bytes;
  const int64_t total = layer_size(layer);
  for (int64_t c = 0; c < int64_t(m.crc.size()); ++c) {
    const int64_t a = c * m.chunk_bytes, b = total > 0 ? std::min(a + m.chunk_bytes, total) : a + m.chunk_bytes;
    bool inside = false;
    for (auto& r : ranges) inside = inside || (r.first <= a && r.second >= b);
    if (inside) pc.second.emplace(c, m.crc[size_t(c)]);
  }
}

void Node::flush_batch() {
  // Assign global sequence numbers: by phase (relay hops after the hops that
  // feed them), then round-robin over (src, dst) pairs so that consecutive
  // sequence numbers spread over distinct xGMI links.
  if (pending_jobs_.empty()) return;
  trace::Scoped tr("dissem.flush_batch");
  std::map<int, std::map<std::pair<NodeID, NodeID>, std::vector<XferJob>>> by_phase;
  for (auto& pj : pending_jobs_) by_phase[pj.phase][{pj.job.src, pj.job.dst}].push_back(pj.job);
  pending_jobs_.clear();
  std::map<NodeID, Message> per_rank;
  for (auto& ph : by_phase) {
    for (size_t round = 0;; ++round) {
      bool any = false;
      for (auto& pr : ph.second) {
        if (round >= pr.second.size()) continue;
        any = true;
        XferJob j = pr.second[round];
        j.seq = next_seq_++;
        per_rank[j.src].jobs.push_back(j);
        if (j.dst == kAllRanks) {
          for (auto& st : status_)
            if (st.first != j.src) per_rank[st.first].jobs.push_back(j);
        } else if (j.dst != j.src) {
          per_rank[j.dst].jobs.push_back(j);
        }
      }
      if (!any) break;
    }
  }
  const uint64_t batch = next_batch_++;
  int64_t njobs = 0;
  for (auto& kv : per_rank) {
    kv.second.type = MsgType::XferBatch;
    kv.second.batch = batch;
    njobs += int64_t(kv.second.jobs.size());
    send_msg(kv.first, kv.second);
  }
  log::debug(int64_t(cfg_.id)).u("batch", batch).i("job_copies", njobs).msg("dispatched transfer batch");
}

void Node::retransmit(LayerID layer, NodeID owner, NodeID dest) {
  // node.go:611-626; the leader's own sends are asynchronous (quirk Q4).
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.jobs_dispatched++;
  }
  if (e_->planned()) {
    add_job(owner, dest, layer, 0, -1);
    return;
  }
  track(owner, dest, layer, 0, layer_size(layer));
  if (owner == cfg_.id) {
    LayerSrc src;
    int64_t rate = store_.get(layer, &src) ? src.meta.limit_rate : 0;
    send_layer(dest, layer, 0, -1, rate);
    return;
  }
  Message r;
  r.type = MsgType::Retransmit;
  r.layer = layer;
  r.dest = dest;
  send_msg(owner, r);
}

void Node::schedule_mode0() {
  // node.go:326-352: the leader pushes every missing (dest, layer) itself.
  std::map<LayerID, std::vector<NodeID>> need;
  for (auto& kv : assignment_)
    for (auto& l : kv.second)
      if (!at(status_[kv.first], l.first, e_->target())) need[l.first].push_back(kv.first);
  int64_t rot = 0;  // relay: which dests take a layer's leftover chunks rotates, so every link carries 1/k
  int64_t srot = 0;  // host_share: which stagers serve a layer with fewer chunks than stagers rotates
  std::map<int, int64_t> host_rot;  // several hosts: which GPUs of a host take the slices rotates
  for (auto& kv : need) {
    LayerSrc src;
    if (!store_.get(kv.first, &src)) {
      log::warn(int64_t(cfg_.id)).msg("no layers found for layerID:" + std::to_string(kv.first));
      continue;
    }
    // host_share (planned engines): every node holding the layer's bytes below
    // HBM (the leader's shared host segment, mapped by each rank) stages one
    // slice of it; the leader is then a dest like any other.
    std::vector<NodeID> stagers;
    const int64_t cb = std::max<int64_t>(e_->chunk_bytes(), 1);
    const int64_t nchunks = (src.data_size + cb - 1) / cb;
    if (cfg_.host_share && e_->planned())
      for (auto& st : status_) {
        auto it = st.second.find(kv.first);
        if (it != st.second.end() && it->second.location != e_->target() && it->second.location != Location::Client)
          stagers.push_back(st.first);
      }
    const bool sliced = stagers.size() >= 2 && nchunks >= 2;
    std::vector<NodeID> remote;
    for (NodeID d : kv.second) {
      if (d == cfg_.id && !sliced) {
        if (e_->planned()) add_job(d, d, kv.first, 0, -1);
        else send_layer(d, kv.first, 0, -1, src.meta.limit_rate);
      } else if (d != cfg_.id) {
        remote.push_back(d);
      }
    }
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.jobs_dispatched += int64_t(kv.second.size());
    }
    if (e_->planned()) {
      const int64_t total = src.data_size;
      bool everyone = cfg_.collective && remote.size() >= 2 && remote.size() + 1 == status_.size();
      if (sliced) {
        // Slice i of the layer is staged by stager i over its own PCIe (a
        // local load if it needs the layer) and sent from its HBM to every
        // other dest; leftover chunks rotate over the stagers layer by layer.
        // A layer of fewer chunks than stagers goes to a rotating subset.
        const int64_t S = int64_t(stagers.size()), k = std::min<int64_t>(S, nchunks);
        int64_t off = 0;
        for (int64_t i = 0; i < k; ++i) {
          const int64_t r = ((i - rot) % k + k) % k;
          const int64_t cnt = nchunks / k + (r < nchunks % k ? 1 : 0);
          const int64_t len = std::min(total - off, cnt * cb);
          if (len <= 0) continue;
          const NodeID s = stagers[size_t((i + srot) % S)];
          for (NodeID d : kv.second) add_job(s, d, kv.first, off, len, 0);
          off += len;
        }
        rot += nchunks % k;
        srot += k;
      } else if (everyone) {
        // Collective: one ncclBroadcast per layer (chunk-pipelined) rooted at the
        // leader; every rank of the communicator takes part.
        add_job(cfg_.id, kAllRanks, kv.first, 0, total, 0);
      } else if (cfg_.relay && remote.size() >= 2 && multi_host()) {
        relay_across_hosts(kv.first, total, remote, host_rot);
      } else if (cfg_.relay && remote.size() >= 2 && total >= int64_t(remote.size()) * cb) {
        // Bandwidth-optimal broadcast on a fully connected xGMI mesh: scatter
        // 1/k of the layer to each of k dests, then every dest relays its share
        // to the other k-1 (per-link load 2/k of the layer instead of 1).
        const int64_t k = int64_t(remote.size());
        int64_t off = 0;
        for (int64_t i = 0; i < k; ++i) {
          // nchunks % k dests get one chunk more; a fixed choice would give the
          // same dests (and their relay links) 3/16 of every 16-chunk layer
          // instead of 1/7 at k = 7
          const int64_t r = ((i - rot) % k + k) % k;
          int64_t cnt = nchunks / k + (r < nchunks % k ? 1 : 0);
          int64_t len = std::min(total - off, cnt * cb);
          add_job(cfg_.id, remote[size_t(i)], kv.first, off, len, 0);
          for (int64_t j = 0; j < k; ++j)
            if (j != i) add_job(remote[size_t(i)], remote[size_t(j)], kv.first, off, len, 1);
          off += len;
        }
        rot += nchunks % k;
      } else {
        for (NodeID d : remote) add_job(cfg_.id, d, kv.first, 0, -1);
      }
    } else if (remote.size() >= 2 && e_->supports_broadcast() && src.meta.location != Location::Client) {
      for (NodeID d : remote) track(cfg_.id, d, kv.first, 0, src.data_size);
      e_->broadcast_layer(kv.first, src.data_size, remote);
    } else {
      for (NodeID d : remote) {
        track(cfg_.id, d, kv.first, 0, src.data_size);
        send_layer(d, kv.first, 0, -1, src.meta.limit_rate);
      }
    }
  }
}

void Node::schedule_mode1() {
  // node.go:554-608: a random current owner retransmits each missing layer.
  for (auto& kv : status_)
    for (auto& l : kv.second) owners_[l.first].insert(kv.first);  // initialized on demand (quirk Q3)
  const bool links = cfg_.owner_policy == "links";
  // Link capacities (config Links / probed topology); unknown links count as
  // the fastest known one, and with none known every link is equal.
  double cap_max = 0;
  for (auto& kv : cfg_.link_bw) cap_max = std::max(cap_max, double(kv.second));
  auto cap = [&](NodeID s, NodeID d) {
    auto it = cfg_.link_bw.find({s, d});
    return it != cfg_.link_bw.end() && it->second > 0 ? double(it->second) : (cap_max > 0 ? cap_max : 1.0);
  };
  RelayPlan plan;
  // Multi-host jobs (planned engines, "links" policy): (host, layer) -> the
  // dests on that host that need the layer and their missing ranges.
  const bool hier = links && e_->planned() && multi_host();
  ImportMap imports;
  for (auto& kv : assignment_) {
    NodeID dest = kv.first;
    for (auto& l : kv.second) {
      LayerID layer = l.first;
      if (at(status_[dest], layer, e_->target())) continue;
      auto oit = owners_.find(layer);
      if (oit != owners_.end() && !oit->second.empty()) {
        if (oit->second.count(dest)) {
          // The dest holds it in a lower tier (disk/host/client): promote locally.
          retransmit(layer, dest, dest);
          continue;
        }
        // Chunk-granular resume: a dest that announced part of this layer (its
        // persisted chunks) loads those ranges locally and receives only the gaps.
        std::vector<std::pair<int64_t, int64_t>> gaps{{0, layer_size(layer)}};
        if (e_->planned()) {
          auto pit = partial_.find(dest);
          auto lit = pit == partial_.end() ? PartialLayers::const_iterator() : pit->second.find(layer);
          if (pit != partial_.end() && lit != pit->second.end() && !lit->second.empty()) {
            gaps.clear();
            int64_t pos = 0;
            for (auto r : lit->second) {
              r.second = std::min(r.second, layer_size(layer));
              if (r.first >= r.second) continue;
              if (r.first > pos) gaps.push_back({pos, r.first});
              {
                std::lock_guard<std::mutex> lk(sig_mu_);
                stats_.jobs_dispatched++;
              }
              add_job(dest, dest, layer, r.first, r.second - r.first);
              pos = std::max(pos, r.second);
            }
            if (pos < layer_size(layer)) gaps.push_back({pos, layer_size(layer)});
            if (gaps.empty()) continue;
          }
        }
        int64_t need = 0;
        for (auto& g : gaps) need += g.second - g.first;
        const bool ranged = gaps.size() != 1 || need != layer_size(layer);
        std::vector<NodeID> cand(oit->second.begin(), oit->second.end());
        if (hier) {
          // Several hosts: a holder on the dest's own host serves it over xGMI;
          // a layer no GPU of that host holds is imported once per host
          // (schedule_imports) instead of once per GPU over the NICs.
          std::vector<NodeID> local;
          for (NodeID c : cand)
            if (host_of(c) == host_of(dest)) local.push_back(c);
          if (local.empty()) {
            imports[{host_of(dest), layer}].push_back({dest, gaps});
            continue;
          }
          cand.swap(local);
        }
        NodeID owner;
        if (links) {
          // xGMI-aware: every GPU pair has its own link, so spread each dest's
          // inbound bytes over distinct links - least projected link time
          // (bytes / capacity) first, then least total egress, then lowest id.
          owner = cand[0];
          std::pair<double, int64_t> best{1e300, INT64_MAX};
          for (NodeID c : cand) {
            std::pair<double, int64_t> k{double(link_bytes_[{c, dest}] + need) / cap(c, dest), owner_bytes_[c]};
            if (k < best) {
              best = k;
              owner = c;
            }
          }
          link_bytes_[{owner, dest}] += need;
        } else if (cfg_.owner_policy == "balanced") {
          int64_t best = INT64_MAX;
          std::vector<NodeID> ties;
          for (NodeID c : cand) {
            int64_t b = owner_bytes_[c];
            if (b < best) {
              best = b;
              ties.assign(1, c);
            } else if (b == best) {
              ties.push_back(c);
            }
          }
          owner = ties[size_t(rng_() % ties.size())];
        } else {
          owner = cand[size_t(rng_() % cand.size())];  // uniform (quirk Q5)
        }
        owner_bytes_[owner] += need;
        if (links && e_->planned()) {
          for (auto& g : gaps) plan[{dest, layer}].push_back(PlanPart{owner, g.first, g.second - g.first, 0});
        } else if (ranged) {
          for (auto& g : gaps) {
            {
              std::lock_guard<std::mutex> lk(sig_mu_);
              stats_.jobs_dispatched++;
            }
            add_job(owner, dest, layer, g.first, g.second - g.first);
          }
        } else {
          retransmit(layer, owner, dest);
        }
      } else {
        LayerSrc src;
        if (!store_.get(layer, &src)) {
          log::warn(int64_t(cfg_.id)).msg("no layers found for layerID:" + std::to_string(layer));
          continue;
        }
        retransmit(layer, cfg_.id, dest);
      }
    }
  }
  if (cap_max > 0 && !plan.empty()) relay_rebalance(plan, cap);
  if (!imports.empty()) schedule_imports(imports, plan, cap);
  if (plan.empty()) return;
  for (auto& kv : plan)
    for (auto& p : kv.second) {
      {
        std::lock_guard<std::mutex> lk(sig_mu_);
        stats_.jobs_dispatched++;
      }
      add_job(p.src, kv.first.first, kv.first.second, p.off, p.size, p.phase);
    }
}

void Node::relay_rebalance(RelayPlan& plan, const std::function<double(NodeID, NodeID)>& cap) {
  // A slow link (config Links / measured topology) must not set the session
  // time: move chunk-sized slices of the layers it carries onto relays. A relay
  // is a rank that receives the same layer straight from an owner in this plan
  // (phase 0); it forwards the slice in phase 1, chunk-pipelined behind its own
  // recv (the planned engine orders a relay after the recv it forwards). Each
  // move takes one slice off the link with the longest projected time onto the
  // relay->dest link whose time stays lowest, while that lowers the maximum.
  const int64_t unit = std::max<int64_t>(cfg_.align, 1);
  std::map<std::pair<NodeID, NodeID>, int64_t> bytes;
  std::set<std::pair<NodeID, LayerID>> relayed_into, relays_from;
  for (auto& kv : plan)
    for (auto& p : kv.second) bytes[{p.src, kv.first.first}] += p.size;
  auto t = [&](NodeID s, NodeID d, int64_t extra) { return double(bytes[{s, d}] + extra) / cap(s, d); };
  int64_t moves = 0;
  for (int iter = 0; iter < 1000000; ++iter) {
    std::pair<NodeID, NodeID> worst{};
    double tw = -1;
    for (auto& kv : bytes)
      if (kv.second > 0 && t(kv.first.first, kv.first.second, 0) > tw) {
        tw = t(kv.first.first, kv.first.second, 0);
        worst = kv.first;
      }
    if (tw <= 0) break;
    const NodeID s = worst.first, d = worst.second;
    bool moved = false;
    for (auto& kv : plan) {
      if (kv.first.first != d || relays_from.count(kv.first)) continue;
      const LayerID layer = kv.first.second;
      auto& parts = kv.second;
      for (size_t i = 0; i < parts.size() && !moved; ++i) {
        PlanPart& p = parts[i];
        if (p.phase != 0 || p.src != s) continue;
        // The slice is the part's last grid chunk: cut on the chunk grid, so an
        // odd layer end moves as one short whole chunk (never two partial
        // pieces of one chunk from different senders).
        const int64_t end = p.off + p.size, cut = (end - 1) / unit * unit;
        if (cut <= p.off) continue;
        const int64_t slice = end - cut;
        // the best relay: receives this layer directly (phase 0 only) in this plan
        NodeID best = 0;
        double tb = 1e300;
        for (auto& other : plan) {
          const NodeID x = other.first.first;
          if (other.first.second != layer || x == d || x == s || relayed_into.count(other.first)) continue;
          if (host_of(x) != host_of(d)) continue;  // relays stay on the dest's host (xGMI)
          const double tx = t(x, d, slice);
          if (tx < tb) {
            tb = tx;
            best = x;
          }
        }
        if (tb >= tw) continue;  // no relay improves on this link
        p.size -= slice;
        parts.push_back(PlanPart{best, cut, slice, 1});
        bytes[{s, d}] -= slice;
        bytes[{best, d}] += slice;
        relayed_into.insert(kv.first);
        relays_from.insert({best, layer});
        moved = true;
        ++moves;
      }
      if (moved) break;
    }
    if (!moved) break;
  }
  if (moves)
    log::info(int64_t(cfg_.id)).i("relayed_slices", moves).i("slice_bytes", unit).msg("mode 1: relays around slow links");
}

void Node::relay_across_hosts(LayerID layer, int64_t total, const std::vector<NodeID>& remote,
                              std::map<int, int64_t>& rot) {
  // Planned mode 0 on several hosts: a three-level broadcast. The leader
  // scatters the layer over its own host's xGMI (one chunk-grid slice per
  // GPU of its host that needs it); each of those GPUs relays its slice to
  // its host peers and forwards it over its NIC to one GPU of every other
  // host, which relays it inside that host. No byte enters a host twice, and
  // the export is spread over the leader host's NICs instead of the leader's
  // one (a flat relay would send every slice into a remote host once per GPU).
  const int64_t cb = std::max<int64_t>(e_->chunk_bytes(), 1), nchunks = (total + cb - 1) / cb;
  const int me = host_of(cfg_.id);
  std::vector<NodeID> local;
  std::map<int, std::vector<NodeID>> far;
  for (NodeID d : remote) (host_of(d) == me ? local : far[host_of(d)]).push_back(d);
  // the GPUs that take the first-level slices: the leader host's dests, or the
  // leader itself when none of its host's GPUs needs the layer
  const bool self_export = local.empty();
  const std::vector<NodeID> tier1 = self_export ? std::vector<NodeID>{cfg_.id} : local;
  const int64_t k = std::max<int64_t>(1, std::min<int64_t>(int64_t(tier1.size()), nchunks));
  int64_t off = 0;
  for (int64_t i = 0; i < k; ++i) {
    const int64_t cnt = nchunks / k + (i < nchunks % k ? 1 : 0);
    const int64_t len = std::min(total - off, cnt * cb);
    if (len <= 0) continue;
    const NodeID a = tier1[size_t((i + rot[me]) % int64_t(tier1.size()))];
    if (!self_export) {
      add_job(cfg_.id, a, layer, off, len, 0);
      for (NodeID d : local)
        if (d != a) add_job(a, d, layer, off, len, 1);
    }
    const int phase = self_export ? 0 : 1;
    for (auto& hv : far) {
      const auto& gpus = hv.second;
      const NodeID entry = gpus[size_t((i + rot[hv.first]) % int64_t(gpus.size()))];
      add_job(a, entry, layer, off, len, phase);
      for (NodeID d : gpus)
        if (d != entry) add_job(entry, d, layer, off, len, phase + 1);
    }
    off += len;
  }
  rot[me] += k;
  for (auto& hv : far) rot[hv.first] += k;
}

int Node::host_of(NodeID n) const {
  auto it = cfg_.host.find(n);
  return it == cfg_.host.end() ? 0 : it->second;
}

bool Node::multi_host() const {
  std::set<int> hosts;
  for (auto& kv : status_) hosts.insert(host_of(kv.first));
  return hosts.size() > 1;
}

void Node::schedule_imports(const ImportMap& imports, RelayPlan& plan,
                            const std::function<double(NodeID, NodeID)>& cap) {
  // Hierarchical dissemination across hosts. A layer that no GPU of host H
  // holds crosses the network once per host, not once per GPU: it is cut on
  // the chunk grid into one slice per dest of H that needs it; slice i goes
  // from a holder on another host to dest i of H over their NICs (phase 0) and
  // dest i relays it to the other dests of H over xGMI (phase 1, chunk-
  // pipelined behind its own recv, as mode 0's scatter + relay). Every GPU's
  // NIC then carries 1/k of each imported layer and its xGMI links the rest.
  // The slice of a layer a dest takes is the next in a rotation over the
  // dests with the least NIC ingress so far; the holder of each slice is the
  // one with the least NIC egress so far (reference: a layer always goes
  // owner -> dest directly, node.go:554-608, which on a multi-node MI355X
  // cluster sends every byte over the NIC once per GPU).
  const int64_t unit = std::max<int64_t>(cfg_.align, 1);
  std::map<NodeID, int64_t> nic_in, nic_out;
  int64_t imported = 0;
  for (auto& kv : imports) {
    const LayerID layer = kv.first.second;
    const int64_t total = layer_size(layer);
    auto oit = owners_.find(layer);
    if (oit == owners_.end() || oit->second.empty()) continue;
    std::vector<NodeID> holders(oit->second.begin(), oit->second.end());
    auto pick_holder = [&](NodeID dest) {
      NodeID best = holders[0];
      std::pair<int64_t, double> bk{INT64_MAX, 1e300};
      for (NodeID h : holders) {
        std::pair<int64_t, double> k{nic_out[h], double(link_bytes_[{h, dest}]) / cap(h, dest)};
        if (k < bk) {
          bk = k;
          best = h;
        }
      }
      return best;
    };
    // Dests missing the whole layer share it by slices; a dest with a partial
    // copy (chunk-granular resume) receives its own gaps directly.
    std::vector<NodeID> whole;
    for (auto& dg : kv.second) {
      const bool full = dg.second.size() == 1 && dg.second[0].first == 0 && dg.second[0].second == total;
      if (full) {
        whole.push_back(dg.first);
        continue;
      }
      for (auto& g : dg.second) {
        const NodeID h = pick_holder(dg.first);
        plan[{dg.first, layer}].push_back(PlanPart{h, g.first, g.second - g.first, 0});
        nic_out[h] += g.second - g.first;
        nic_in[dg.first] += g.second - g.first;
        link_bytes_[{h, dg.first}] += g.second - g.first;
      }
    }
    if (whole.empty()) continue;
    const int64_t nchunks = (total + unit - 1) / unit;
    const int64_t k = std::min<int64_t>(int64_t(whole.size()), std::max<int64_t>(nchunks, 1));
    // entries: the k dests with the least NIC ingress so far take the slices
    std::stable_sort(whole.begin(), whole.end(), [&](NodeID a, NodeID b) { return nic_in[a] < nic_in[b]; });
    int64_t off = 0;
    for (int64_t i = 0; i < k; ++i) {
      const int64_t cnt = nchunks / k + (i < nchunks % k ? 1 : 0);
      const int64_t len = std::min(total - off, cnt * unit);
      if (len <= 0) continue;
      const NodeID entry = whole[size_t(i)];
      const NodeID h = pick_holder(entry);
      plan[{entry, layer}].push_back(PlanPart{h, off, len, 0});
      nic_out[h] += len;
      nic_in[entry] += len;
      link_bytes_[{h, entry}] += len;
      for (NodeID d : whole)
        if (d != entry) {
          plan[{d, layer}].push_back(PlanPart{entry, off, len, 1});
          link_bytes_[{entry, d}] += len;
        }
      off += len;
    }
    imported++;
  }
  if (imported)
    log::info(int64_t(cfg_.id)).i("imported_layer_copies", imported).msg("mode 1: layers imported once per host, relayed over xGMI");
}

// ------------------------------------------------------------------- mode 2

NodeID Node::min_loaded_sender(LayerID layer, NodeID dest) {
  // node.go:948-978 (the code picks the FASTEST source; quirk Q16 keeps that).
  // A sender's rate for this job is its tier's LimitRate capped by its link to
  // the dest when the plan knows it (measured or configured): on equal links
  // this is the reference's choice.
  // A dest that holds the layer in another tier loads it itself (as modes 1
  // and 3 do): a transfer from a peer would land on top of its own staging
  // of the same chunks (a race TSAN caught in the rank-death selftest).
  if (!suspects_.count(dest)) {
    auto sd = status_.find(dest);
    if (sd != status_.end() && sd->second.count(layer) && load_.count(dest)) return dest;
  }
  // Several hosts: a holder on the dest's host (xGMI) before any across the
  // network (the NIC a GPU shares with all of its remote peers).
  NodeID best = 0;
  bool found = false, best_local = false;
  int64_t best_rate = 0;
  int64_t min_count = INT64_MAX;
  for (auto& kv : load_) {
    NodeID sender = kv.first;
    if (suspects_.count(sender)) continue;  // missed a deadline: no new work
    auto st = status_.find(sender);
    if (st == status_.end()) continue;
    auto it = st->second.find(layer);
    if (it == st->second.end()) continue;
    int64_t eff = it->second.limit_rate == 0 ? INT64_MAX : it->second.limit_rate;
    if (auto lb = cfg_.link_bw.find({sender, dest}); lb != cfg_.link_bw.end() && lb->second > 0 && sender != dest)
      eff = std::min(eff, lb->second);
    int64_t count = kv.second;
    const bool local = host_of(sender) == host_of(dest);
    if (!found || (local && !best_local) ||
        (local == best_local &&
         (eff > best_rate || (eff == best_rate && (count < min_count || (count == min_count && sender < best)))))) {
      best = sender;
      best_rate = eff;
      min_count = count;
      best_local = local;
      found = true;
    }
  }
  return found ? best : kClientID;
}

bool Node::rarest_own_job(NodeID node, LayerID* layer, JobKey* key) {
  // node.go:981-1010 (ties: lowest layer id, then lowest (dest, offset))
  bool ok = false;
  size_t min_owners = SIZE_MAX;
  auto st = status_.find(node);
  if (st == status_.end()) return false;
  for (auto& l : st->second) {
    auto lj = jobs_.find(l.first);
    if (lj == jobs_.end()) continue;
    for (auto& jd : lj->second) {
      if (jd.second.sender != node || jd.second.state != JobState::Pending) continue;
      size_t cnt = owners_[l.first].size();
      if (!ok || cnt < min_owners || (cnt == min_owners && l.first < *layer)) {
        min_owners = cnt;
        *layer = l.first;
        *key = jd.first;
        ok = true;
      }
    }
  }
  return ok;
}

bool Node::rarest_stealable_job(NodeID node, LayerID* layer, JobKey* key, NodeID* victim) {
  // node.go:1012-1073
  struct Cand {
    LayerID layer;
    JobKey dest;
    NodeID sender;
    size_t owners;
    double ttf;
  };
  bool have = false;
  Cand best{};
  auto st = status_.find(node);
  if (st == status_.end()) return false;
  for (auto& l : st->second) {
    auto lj = jobs_.find(l.first);
    if (lj == jobs_.end()) continue;
    size_t cnt = owners_[l.first].size();
    for (auto& jd : lj->second) {
      NodeID sender = jd.second.sender;
      int64_t sender_rate = 0;
      if (auto s2 = status_.find(sender); s2 != status_.end())
        if (auto x = s2->second.find(l.first); x != s2->second.end()) sender_rate = x->second.limit_rate;
      int64_t node_rate = l.second.limit_rate;
      if (sender == node || jd.second.state != JobState::Pending || load_[sender] == 0 ||
          (node_rate != 0 && node_rate < sender_rate))
        continue;
      // several hosts: a job its dest's own host serves (xGMI) is not stolen across the network
      const NodeID dest = jd.first.first;
      if (host_of(node) != host_of(dest) && host_of(sender) == host_of(dest) && multi_host()) continue;
      double ttf = perf_.count(sender) ? perf_[sender].first * double(load_[sender]) : 1e300;
      Cand c{l.first, jd.first, sender, cnt, ttf};
      if (!have || c.owners < best.owners || (c.owners == best.owners && c.ttf > best.ttf)) {
        best = c;
        have = true;
      }
    }
  }
  if (!have) return false;
  *layer = best.layer;
  *key = best.dest;
  *victim = best.sender;
  return true;
}

void Node::dispatch_range(LayerID layer, NodeID sender, NodeID dest, int64_t off, int64_t size) {
  if (off == 0 && size >= layer_size(layer)) {
    retransmit(layer, sender, dest);  // whole layer: the reference's Retransmit
    return;
  }
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.jobs_dispatched++;
  }
  if (e_->planned()) {
    add_job(sender, dest, layer, off, size);
    return;
  }
  track(sender, dest, layer, off, size);
  if (sender == cfg_.id) {
    send_layer(dest, layer, off, size, 0);
    return;
  }
  Message f;  // a byte range: FlowRetransmit carries offset + size
  f.type = MsgType::FlowRetransmit;
  f.layer = layer;
  f.dest = dest;
  f.offset = off;
  f.data_size = size;
  send_msg(sender, f);
}

bool Node::assign_new_job(NodeID node) {
  // node.go:909-945
  LayerID layer = 0;
  JobKey key{0, 0};
  NodeID victim = 0;
  if (suspects_.count(node)) return false;
  if (rarest_own_job(node, &layer, &key)) {
    Job& j = jobs_[layer][key];
    j.state = JobState::Sending;
    j.t_us = log::now_us();
    load_[node] = std::max<int64_t>(0, load_[node] - 1);
    inflight_[node]++;
    log::debug(int64_t(cfg_.id)).u("node", node).u("layer", layer).i("offset", key.second)
        .msg("pass a job initially assigned");
    dispatch_range(layer, node, key.first, key.second, j.size);
    return true;
  }
  if (rarest_stealable_job(node, &layer, &key, &victim)) {
    log::debug(int64_t(cfg_.id)).u("layer", layer)
        .msg("steal a job from the most loaded node (" + std::to_string(victim) + ") to node " + std::to_string(node));
    load_[victim] = std::max<int64_t>(0, load_[victim] - 1);
    Job& j = jobs_[layer][key];
    j.sender = node;
    j.state = JobState::Sending;
    j.t_us = log::now_us();
    inflight_[node]++;
    dispatch_range(layer, node, key.first, key.second, j.size);
    return true;
  }
  log::debug(int64_t(cfg_.id)).u("node", node).msg("there is no job left to assign");
  return false;
}

void Node::schedule_mode2() {
  // node.go:810-904
  for (auto& kv : status_)
    for (auto& l : kv.second) owners_[l.first].insert(kv.first);
  std::vector<LayerID> sorted;
  for (auto& kv : owners_) sorted.push_back(kv.first);
  std::stable_sort(sorted.begin(), sorted.end(), [&](LayerID a, LayerID b) {
    if (owners_[a].size() != owners_[b].size()) return owners_[a].size() < owners_[b].size();
    return a < b;  // rarest first, tiebreak by id
  });
  // Jobs are (layer, dest, range). With pull_job_bytes the layer is cut into
  // ranges (chunk-aligned on planned engines) so stealing can rebalance inside
  // a layer; 0 keeps the reference's one job per (layer, dest).
  int64_t jb = cfg_.pull_job_bytes;
  if (jb > 0 && e_->planned() && e_->chunk_bytes() > 0)
    jb = std::max<int64_t>(1, (jb + e_->chunk_bytes() - 1) / e_->chunk_bytes()) * e_->chunk_bytes();
  for (auto& kv : assignment_)
    for (auto& l : kv.second) {
      if (at(status_[kv.first], l.first, e_->target())) continue;
      const int64_t size = layer_size(l.first);
      const int64_t step = jb > 0 ? jb : std::max<int64_t>(size, 1);
      for (int64_t off = 0; off < std::max<int64_t>(size, 1); off += step) {
        Job j;
        j.size = std::min(step, size - off);
        jobs_[l.first][{kv.first, off}] = j;
      }
    }
  for (auto& kv : status_) load_.emplace(kv.first, 0);
  // Several hosts (planned engines): a layer that no GPU of a host holds is
  // pulled across the network by one GPU of that host - the entry, the dest
  // with the fewest imports so far - and every other dest of the host pulls it
  // from the entry once it holds it (its ack makes it an owner and kicks it),
  // over xGMI. Jobs from an entry are not stolen across hosts.
  const bool hier = e_->planned() && multi_host();
  std::map<std::pair<int, LayerID>, NodeID> entry;
  if (hier) {
    std::map<NodeID, int> imports;
    for (LayerID layer : sorted) {
      auto lj = jobs_.find(layer);
      if (lj == jobs_.end()) continue;
      std::map<int, std::set<NodeID>> remote_dests;  // host -> dests with no holder on it
      for (auto& jd : lj->second) {
        const NodeID d = jd.first.first;
        const NodeID s = min_loaded_sender(layer, d);
        if (s != kClientID && host_of(s) != host_of(d)) remote_dests[host_of(d)].insert(d);
      }
      for (auto& hv : remote_dests) {
        NodeID e = *hv.second.begin();
        for (NodeID d : hv.second)
          if (imports[d] < imports[e]) e = d;
        imports[e]++;
        entry[{hv.first, layer}] = e;
      }
    }
  }
  for (LayerID layer : sorted) {
    auto lj = jobs_.find(layer);
    if (lj == jobs_.end()) continue;
    for (auto& jd : lj->second) {
      NodeID sender = min_loaded_sender(layer, jd.first.first);
      if (sender == kClientID) {
        log::error(int64_t(cfg_.id)).u("layer", layer).msg("no owner holds the layer");
        continue;
      }
      if (hier && host_of(sender) != host_of(jd.first.first)) {
        auto en = entry.find({host_of(jd.first.first), layer});
        if (en != entry.end() && en->second != jd.first.first) sender = en->second;
      }
      jd.second.sender = sender;
      jd.second.state = JobState::Pending;
      load_[sender]++;
      log::info(int64_t(cfg_.id)).msg("job assignment: layer: " + std::to_string(layer) +
                                      ", sender: " + std::to_string(sender));
    }
  }
  // Kick every node that has queued jobs or is a destination (quirk Q10:
  // the reference kicks only assignment keys, stranding pure senders).
  std::set<NodeID> kick;
  for (auto& kv : assignment_) kick.insert(kv.first);
  for (auto& kv : load_)
    if (kv.second > 0) kick.insert(kv.first);
  for (NodeID n : kick)
    while (inflight_[n] < cfg_.pull_window && assign_new_job(n)) {
    }
}

// ------------------------------------------------------------------- mode 3

void Node::schedule_mode3() {
  // node.go:1200-1288 + flow.go
  FlowProblem p;
  const Location tgt = e_->target();
  std::vector<FlowDemand> demands;
  struct SelfJob {
    NodeID dest;
    LayerID layer;
    int64_t size, rate;
  };
  std::vector<SelfJob> self_jobs;
  for (auto& kv : assignment_) {
    for (auto& l : kv.second) {
      auto& st = status_[kv.first];
      if (at(st, l.first, tgt)) continue;
      auto it = st.find(l.first);
      if (it != st.end()) {
        self_jobs.push_back({kv.first, l.first, layer_size(l.first), it->second.limit_rate});
      } else {
        demands.push_back({l.first, kv.first, layer_size(l.first)});
      }
    }
  }
  for (auto& sj : self_jobs) {
    Message f;
    f.type = MsgType::FlowRetransmit;
    f.layer = sj.layer;
    f.dest = sj.dest;
    f.data_size = sj.size;
    f.offset = 0;
    f.rate = sj.rate;
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.jobs_dispatched++;
    }
    if (e_->planned()) {
      add_job(sj.dest, sj.dest, sj.layer, 0, sj.size);
    } else {
      track(sj.dest, sj.dest, sj.layer, 0, sj.size);
      send_msg(sj.dest, f);
    }
  }
  if (demands.empty()) {
    log::info(int64_t(cfg_.id)).msg("No jobs to assign other than self-assignment");
    return;
  }
  p.demands = demands;
  p.holdings = status_;
  for (auto& kv : cfg_.network_bw) {
    p.egress_bps[kv.first] = kv.second;
    p.ingress_bps[kv.first] = kv.second;
  }
  for (auto& kv : cfg_.hbm_bw) {
    if (kv.second <= 0) continue;
    auto it = p.ingress_bps.find(kv.first);
    if (it == p.ingress_bps.end() || it->second <= 0 || it->second > kv.second) p.ingress_bps[kv.first] = kv.second;
  }
  p.link_bps = cfg_.link_bw;
  p.stage_bps = cfg_.stage_bw;
  p.align = cfg_.align;
  p.integer_seconds = cfg_.integer_seconds;
  p.disk_group = cfg_.disk_group;
  p.disk_group_bps = cfg_.disk_group_bw;
  if (multi_host()) {
    p.host = cfg_.host;
    p.nic_bps = cfg_.nic_bw;
  }
  if (e_->planned()) {
    // GPU data plane: a layer is loaded into HBM once and forwarded from there;
    // a self-job's load feeds the dest's own sends of that layer too.
    p.stage_once = true;
    for (auto& sj : self_jobs) {
      auto st = status_[sj.dest].find(sj.layer);
      if (st != status_[sj.dest].end() && st->second.source_type != SourceType::Device)
        p.self_loads[sj.dest][sj.layer] = sj.size;
    }
  }
  log::info(int64_t(cfg_.id)).msg("assigning a job...");
  int64_t t0 = log::now_us();
  FlowPlan plan = solve_flow(p);
  if (!plan.feasible && plan.solver == "lp") {
    // The LP did not solve (numerics on extreme measured rates, or its pivot
    // limit): plan with the flow instead - it relaxes the budgets it cannot
    // state, so its T may be optimistic, but every demand gets a sender.
    log::warn(int64_t(cfg_.id)).s("lp_status", plan.lp_status).i("lp_pivots", plan.lp_pivots)
        .msg("mode 3: the LP failed, planning with the max-flow instead");
    p.solver = "flow";
    plan = solve_flow(p);
  }
  log::info(int64_t(cfg_.id)).f("computation time[ms]", double(log::now_us() - t0) / 1e3).i("solves", plan.solves)
      .s("solver", plan.solver).i("lp_pivots", plan.lp_pivots).msg("Job assignment completed");
  log::info(int64_t(cfg_.id)).f("required minimum time(s)", plan.T).b("feasible", plan.feasible)
      .msg("job assignment calculated");
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.flow_T = plan.T;
  }
  // Safety net: every demand's byte ranges must cover the layer, or its dest
  // never completes it and the session hangs. A plan that leaves a gap (the
  // LP's rounding of tiny shares onto the chunk grid can) gets the gap from
  // the demand's largest sender, at the plan's pace.
  if (plan.feasible) {
    std::map<std::pair<LayerID, NodeID>, std::vector<std::pair<int64_t, int64_t>>> cover;
    std::map<std::pair<LayerID, NodeID>, std::pair<NodeID, int64_t>> biggest;
    for (auto& j : plan.jobs) {
      cover[{j.layer, j.dest}].push_back({j.offset, j.offset + j.size});
      auto& b = biggest[{j.layer, j.dest}];
      if (j.size > b.second) b = {j.sender, j.size};
    }
    int64_t filled = 0;
    for (auto& d : p.demands) {
      auto& v = cover[{d.layer, d.dest}];
      std::sort(v.begin(), v.end());
      int64_t pos = 0;
      std::vector<std::pair<int64_t, int64_t>> gaps;
      for (auto& r : v) {
        if (r.first > pos) gaps.push_back({pos, r.first});
        pos = std::max(pos, r.second);
      }
      if (pos < d.size) gaps.push_back({pos, d.size});
      auto bg = biggest.find({d.layer, d.dest});
      NodeID src = bg != biggest.end() ? bg->second.first : kClientID;
      if (src == kClientID)
        for (auto& hs : p.holdings)
          if (hs.first != d.dest && hs.second.count(d.layer)) {
            src = hs.first;
            break;
          }
      if (src == kClientID) continue;
      for (auto& g : gaps) {
        plan.jobs.push_back(FlowJob{src, d.layer, d.dest, g.second - g.first, g.first});
        filled += g.second - g.first;
      }
    }
    if (filled)
      log::warn(int64_t(cfg_.id)).i("gap_bytes", filled).msg("mode 3: the plan left bytes uncovered; filled from a sender");
  }
  for (auto& j : plan.jobs) {
    Message f;
    f.type = MsgType::FlowRetransmit;
    f.layer = j.layer;
    f.dest = j.dest;
    f.data_size = j.size;
    f.offset = j.offset;
    f.rate = plan.T > 0 ? int64_t(double(j.size) / plan.T) : 0;  // node.go:1281 (pace to finish together)
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.jobs_dispatched++;
    }
    if (e_->planned()) {
      add_job(j.sender, j.dest, j.layer, j.offset, j.size, 0, f.rate);
    } else {
      track(j.sender, j.dest, j.layer, j.offset, j.size);
      send_msg(j.sender, f);
    }
  }
}

// ------------------------------------------------------------------- client

ClientNode::ClientNode(NodeID node_id, std::shared_ptr<Transport> t, const LayersSrc& layers)
    : node_id_(node_id), t_(std::move(t)), layers_(layers) {}

ClientNode::~ClientNode() { stop(); }

void ClientNode::start() {
  th_ = std::thread([this] {
    for (;;) {
      auto m = t_->deliver().pop();
      if (!m || (*m)->type == MsgType::Stop) break;
      if ((*m)->type != MsgType::ClientReq) continue;
      LayerID layer = (*m)->layer;
      auto it = layers_.find(layer);
      if (it == layers_.end() || !it->second.host) {
        log::error(-1).u("layerID", layer).msg("client does not hold the layer");
        continue;
      }
      LayerSrc src = it->second;
      workers_.spawn([this, layer, src] {
        // client.go:48-63: stream the whole layer to the attached node.
        Message lm;
        lm.type = MsgType::Layer;
        lm.src = kClientID;
        lm.layer = layer;
        lm.data_size = src.data_size;
        lm.total_size = src.data_size;
        lm.offset = 0;
        lm.rate = src.meta.limit_rate;
        LayerPayload p;
        p.host = src.host;
        try {
          t_->send(node_id_, lm, &p);
        } catch (const std::exception& e) {
          log::error(-1).s("error", e.what()).msg("failed to send layer to " + std::to_string(node_id_));
        }
      });
    }
  });
}

void ClientNode::stop() {
  if (!th_.joinable()) return;
  auto m = std::make_shared<Message>();
  m->type = MsgType::Stop;
  t_->inject(m);
  th_.join();
  workers_.join_all();
}

}  // namespace dissem
