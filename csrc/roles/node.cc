#include "roles/node.h"
#include "roles/node_internal.h"
#include "roles/plan_cache.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <set>
#include <thread>
#include <tuple>

#include "core/log.h"
#include "core/trace.h"
#include "sched/maxflow.h"

namespace dissem {


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
    merge_link_rates(cfg_.id, cfg_.link_report, cfg_.link_report_in);
  }
  e_->bind(this);
  if (is_leader_ && e_->planned()) {
    // Whole copies only, the filter announce() applies: a resumed partial copy's
    // manifest holds CRC 0 for every chunk it lacks. Its real chunks are merged
    // per chunk (merge_partial_manifest), like any other partial holder's.
    const LayerIDs inv = store_.inventory();
    const PartialLayers part = store_.partial();
    for (auto& kv : e_->manifest()) {
      if (inv.count(kv.first)) {
        manifests_[kv.first] = kv.second;
        manifest_holders_[kv.first].insert(cfg_.id);
      }
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
  loop_th_ = vclock::spawn([this] { loop(); }, "node-loop");
  if (is_leader_) {
    // A leader whose assignment names only itself gets no announce: check once at start.
    auto m = std::make_shared<Message>();
    m->type = MsgType::Tick;
    m->epoch = cfg_.epoch;
    t_->inject(m);
    if (cfg_.job_timeout_s > 0) tick_th_ = vclock::spawn([this] { ticker(); }, "node-tick");
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
  m.link_rates_in = cfg_.link_report_in;
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

// A directed link s -> d is timed at both ends: s reports it with its send
// rates, d with its receive rates (the announces arrive in any order).
void Node::merge_link_rates(NodeID src, const std::map<NodeID, int64_t>& out, const std::map<NodeID, int64_t>& in) {
  for (auto& kv : out) reported_out_[{src, kv.first}] = kv.second;
  for (auto& kv : in) reported_in_[{kv.first, src}] = kv.second;
}

// The rate a link is planned on. Each end's P2P time includes waiting for the
// other end to post, so normally the FASTER reading is the link's (the later
// poster timed the transfer alone: a late receiver must not read as a slow
// link). But a rank reports one level for all its normal links
// (Runtime.link_report), so a node whose egress is slow on EVERY link reports
// a low level while each receiver still reports its own (fast) level until it
// has flagged the link over LINK_SLOW_SESSIONS sessions: the faster reading
// would hide it. A node whose level lies below kSlowNode of the median level
// of its direction is such a node: its links plan on the SLOWER reading.
void Node::merged_link_rates() {
  constexpr double kSlowNode = 0.7;  // Runtime.LINK_SLOW
  auto levels = [](const std::map<std::pair<NodeID, NodeID>, int64_t>& rep, bool by_src) {
    std::map<NodeID, std::vector<int64_t>> per;
    for (auto& kv : rep)
      if (kv.second > 0) per[by_src ? kv.first.first : kv.first.second].push_back(kv.second);
    std::map<NodeID, int64_t> lvl;
    for (auto& kv : per) {
      std::sort(kv.second.begin(), kv.second.end());
      lvl[kv.first] = kv.second[kv.second.size() / 2];
    }
    return lvl;
  };
  auto slow_nodes = [&](const std::map<NodeID, int64_t>& lvl) {
    std::vector<int64_t> v;
    for (auto& kv : lvl) v.push_back(kv.second);
    std::set<NodeID> slow;
    if (v.empty()) return slow;
    std::sort(v.begin(), v.end());
    const double med = double(v[v.size() / 2]);
    for (auto& kv : lvl)
      if (double(kv.second) < kSlowNode * med) slow.insert(kv.first);
    return slow;
  };
  const std::set<NodeID> slow_out = slow_nodes(levels(reported_out_, true));
  const std::set<NodeID> slow_in = slow_nodes(levels(reported_in_, false));
  measured_links_.clear();
  for (auto& kv : reported_out_) measured_links_[kv.first] = kv.second;
  for (auto& kv : reported_in_) {
    auto it = measured_links_.find(kv.first);
    if (it == measured_links_.end()) {
      measured_links_[kv.first] = kv.second;
    } else if (slow_out.count(kv.first.first) || slow_in.count(kv.first.second)) {
      it->second = std::min(it->second, kv.second);
    } else {
      it->second = std::max(it->second, kv.second);
    }
  }
}

void Node::on_announce(const MessagePtr& m) {
  // node.go:295-324
  if (!status_.count(m->src)) {
    std::lock_guard<std::mutex> lk(sig_mu_);
    status_[m->src] = m->layers;
    partial_[m->src] = m->partial_layers;
    add_node(m->src);
    merge_link_rates(m->src, m->link_rates, m->link_rates_in);
  }
  if (!started_) t_->warm(m->src);  // the first dispatch after "timer start" pays no connect
  for (auto& kv : m->manifest) {
    auto pit = m->partial_layers.find(kv.first);
    if (pit != m->partial_layers.end()) {  // a partial copy vouches for its own chunks only
      merge_partial_manifest(kv.first, kv.second, pit->second);
      continue;
    }
    manifest_holders_[kv.first].insert(m->src);
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

namespace {
struct KeyWriter {
  std::string& s;
  template <class T>
  void put(const T& v) {
    s.append(reinterpret_cast<const char*>(&v), sizeof v);
  }
  void put(const std::string& v) {
    put(uint64_t(v.size()));
    s.append(v);
  }
  template <class K, class V>
  void put(const std::map<K, V>& m) {
    put(uint64_t(m.size()));
    for (auto& kv : m) {
      put(kv.first);
      put(kv.second);
    }
  }
  template <class A, class B>
  void put(const std::pair<A, B>& p) {
    put(p.first);
    put(p.second);
  }
  template <class T>
  void put(const std::vector<T>& v) {
    put(uint64_t(v.size()));
    for (auto& x : v) put(x);
  }
  template <class T>
  void put(const std::set<T>& v) {
    put(uint64_t(v.size()));
    for (auto& x : v) put(x);
  }
  void put(const LayerMeta& m) {
    put(int(m.location));
    put(m.limit_rate);
    put(int(m.source_type));
    put(m.size);
  }
  void put(const CrcManifest& m) {
    put(m.chunk_bytes);
    put(m.crc);
  }
};
}  // namespace

// Everything a deterministic scheduler reads, as bytes (roles/plan_cache.h).
std::string Node::plan_key() {
  std::string s;
  s.reserve(64 << 10);
  KeyWriter w{s};
  w.put(cfg_.mode);
  w.put(cfg_.id);
  w.put(cfg_.owner_policy);
  w.put(cfg_.align);
  w.put(cfg_.integer_seconds);
  w.put(cfg_.relay);
  w.put(cfg_.collective);
  w.put(cfg_.host_share);
  w.put(e_->chunk_bytes());
  w.put(int(e_->target()));
  w.put(cfg_.network_bw);
  w.put(cfg_.link_bw);
  w.put(cfg_.stage_bw);
  w.put(cfg_.hbm_bw);
  w.put(cfg_.disk_group);
  w.put(cfg_.disk_group_bw);
  w.put(cfg_.host);
  w.put(cfg_.nic_bw);
  w.put(status_);
  w.put(partial_);
  w.put(assignment_);
  w.put(manifests_);
  w.put(uint64_t(partial_crc_.size()));
  for (auto& kv : partial_crc_) {
    w.put(kv.first);
    w.put(kv.second.first);
    w.put(kv.second.second);
  }
  return s;
}

void Node::start_distribution() {
  int64_t planned = 0;
  for (auto& kv : assignment_)
    for (auto& l : kv.second)
      if (!at(status_[kv.first], l.first, e_->target())) planned += layer_size(l.first);
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    started_ = true;
    t_start_us_ = vclock::now_us();
    stats_.bytes_planned = planned;
    sig_cv_.notify_all();
  }
  initial_status_ = status_;
  merged_link_rates();
  if (cfg_.adapt_links && !measured_links_.empty()) {
    // Closed loop: plan on the capacities the senders measured (reported with
    // their announces) instead of the estimates; links nobody measured keep
    // theirs. Each rank reports one level for all its normal links and its own
    // rate only for a persistently slow one (Runtime.link_report); levels within
    // kLevelSnap of the median report plan as that median, so the ranks' small
    // differences never reshape a uniform plan (and an unchanged fabric gives
    // an unchanged plan: roles/plan_cache.h).
    constexpr double kLevelSnap = 0.15;
    std::vector<int64_t> v;
    for (auto& kv : measured_links_)
      if (kv.second > 0) v.push_back(kv.second);
    if (!v.empty()) {
      std::sort(v.begin(), v.end());
      const int64_t med = v[v.size() / 2];
      std::lock_guard<std::mutex> lk(sig_mu_);
      for (auto& kv : measured_links_)
        if (kv.second > 0)
          cfg_.link_bw[kv.first] = std::abs(double(kv.second - med)) <= kLevelSnap * double(med) ? med : kv.second;
    }
  }
  log::info(int64_t(cfg_.id)).i("mode", cfg_.mode).i("bytes_planned", planned)
      .i("measured_links", int64_t(measured_links_.size())).msg("timer start");
  session_range_ = trace::start("dissem.session");
  int64_t t0 = log::now_us();
  {
    trace::Scoped plan("dissem.plan");
    // Deterministic schedulers on the planned data plane replay an identical
    // earlier plan (roles/plan_cache.h).
    const bool cacheable = e_->planned() && ((cfg_.mode == 1 && cfg_.owner_policy == "links") || cfg_.mode == 3);
    std::string key;
    std::shared_ptr<const CachedPlan> hit;
    if (cacheable) {
      key = plan_key();
      hit = PlanCache::instance().get(key);
    }
    if (hit) {
      pending_jobs_.reserve(hit->jobs.size());
      for (auto& j : hit->jobs) pending_jobs_.push_back({j.first, j.second});
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.jobs_dispatched += hit->dispatched;
      stats_.flow_T = hit->flow_T;
      stats_.plan_solver = hit->solver;
      stats_.plan_cached = true;
    } else {
      const int64_t d0 = stats_.jobs_dispatched;
      {
        std::lock_guard<std::mutex> lk(sig_mu_);
        stats_.plan_solver = cfg_.mode == 1 ? "mode1:" + cfg_.owner_policy : "mode" + std::to_string(cfg_.mode);
      }
      switch (cfg_.mode) {
        case 0: schedule_mode0(); break;
        case 1: schedule_mode1(); break;
        case 2: schedule_mode2(); break;
        case 3: schedule_mode3(); break;
        default: log::error(int64_t(cfg_.id)).msg("unknown mode");
      }
      if (cacheable) {
        CachedPlan cp;
        for (auto& pj : pending_jobs_) cp.jobs.push_back({pj.job, pj.phase});
        std::lock_guard<std::mutex> lk(sig_mu_);
        cp.dispatched = stats_.jobs_dispatched - d0;
        cp.flow_T = stats_.flow_T;
        cp.solver = stats_.plan_solver;
        PlanCache::instance().put(key, std::move(cp));
      }
    }
    const int64_t t1 = log::now_us();
    flush_batch();
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.plan_sched_ms = double(t1 - t0) / 1e3;
    stats_.plan_dispatch_ms = double(log::now_us() - t1) / 1e3;
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
      t_ready_us_ = vclock::now_us();
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
  while (assign_new_job(m->src)) {
  }
  flush_batch();
}

void Node::finish_if_satisfied() {
  if (satisfied_ || !assignment_satisfied()) return;
  // Fire exactly once (quirk Q13).
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    satisfied_ = true;
    t_ready_us_ = vclock::now_us();
    stats_.time_to_deliver_s = double(t_ready_us_ - t_start_us_) / 1e6;
  }
  log::info(int64_t(cfg_.id)).f("time_to_deliver_s", stats_.time_to_deliver_s).msg("timer stop: startup");
  trace::stop(session_range_);
  send_startup();
  std::lock_guard<std::mutex> lk(sig_mu_);
  sig_cv_.notify_all();
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
