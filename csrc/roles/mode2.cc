// Mode 2: pull-retransmit scheduler (reference: node.go:628-1073) - rarest-first
// jobs, min-load initial senders, work stealing by throughput, extended to
// byte-range jobs and a per-sender window.
#include "roles/node.h"

#include <algorithm>
#include <climits>
#include <set>
#include <tuple>

#include "core/log.h"
#include "core/trace.h"
#include "roles/node_internal.h"

namespace dissem {

// ------------------------------------------------------------------- mode 2

NodeID Node::min_loaded_sender(LayerID layer, NodeID dest) {
  // node.go:948-978 (the code picks the FASTEST source; quirk Q16 keeps that).
  // A sender's rate for this job is its tier's LimitRate capped by its link to
  // the dest when the plan knows it (measured or configured): on equal links
  // this is the reference's choice.
  // Planned (GPU) engines: a dest that holds the layer in another tier loads
  // it itself (as modes 1 and 3 do): a peer's transfer into the same HBM slot
  // would race the dest's own staging of those chunks (TSAN caught it in the
  // rank-death selftest). Host engines keep the reference's choice below, the
  // dest competing with its tier rate like any sender (node.go:948-978).
  if (e_->planned() && !suspects_.count(dest)) {
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

// Planned engines: a sender's loads of its own layers (sender == dest, the
// min_loaded_sender choice for a dest holding a layer in another tier) take no
// network window slot - they stage over PCIe, not a link - but have a window
// of two of their own (one layer loading while the last one's check and ack
// complete), so the rest stay pending (stealable by a faster peer)
// and a sender's links always have pull_window jobs queued: with the loads in
// the network window, a lane at N = 2 waited one chunk's staging per layer for
// its next job (sim with the verify model: 910 vs 862 ms, bound 859). The
// engine keeps such loads from queueing whole layers ahead of its sends
// (PlannedEngine kPromoteAhead). Host engines count every job in one window,
// as the reference pulls one job per sender (node.go:764-807).
constexpr int kSelfWindow = 2;

bool Node::job_room(NodeID sender, NodeID dest) {
  if (self_job(sender, dest)) return self_inflight_[sender] < kSelfWindow;
  return inflight_[sender] < cfg_.pull_window;
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
      if (!job_room(node, jd.first.first)) continue;
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
      // a slower node never steals (node.go:1037-1043 skips nodeRate < senderRate);
      // 0 = unlimited on both sides (quirk Q1: the reference let a limited node
      // steal from an unlimited one, whose rate reads 0)
      auto eff = [](int64_t r) { return r == 0 ? INT64_MAX : r; };
      if (sender == node || jd.second.state != JobState::Pending || load_[sender] == 0 ||
          eff(node_rate) < eff(sender_rate))
        continue;
      const NodeID dest = jd.first.first;
      if (!job_room(node, dest)) continue;
      // A dest's own load of a layer it holds (sender == dest) is stolen like
      // any job (node.go:1036-1042): e.g. a peer holding it in memory relieves
      // a dest reading it from a slow tier. If that dest also stages the chunks
      // (for its own sends), the peer's copy lands in scratch (PlannedEngine
      // issue_lane), never a second time into the live slot.
      // several hosts: a job its dest's own host serves (xGMI) is not stolen across the network
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

bool Node::assign_new_job(NodeID node, bool steal) {
  // node.go:909-945
  LayerID layer = 0;
  JobKey key{0, 0};
  NodeID victim = 0;
  if (suspects_.count(node)) return false;
  if (rarest_own_job(node, &layer, &key)) {
    Job& j = jobs_[layer][key];
    j.state = JobState::Sending;
    j.t_us = vclock::now_us();
    load_[node] = std::max<int64_t>(0, load_[node] - 1);
    job_slots(node, key.first)++;
    log::debug(int64_t(cfg_.id)).u("node", node).u("dest", key.first).u("layer", layer).i("offset", key.second)
        .msg("pass a job initially assigned");
    dispatch_range(layer, node, key.first, key.second, j.size);
    return true;
  }
  if (steal && rarest_stealable_job(node, &layer, &key, &victim)) {
    log::debug(int64_t(cfg_.id)).u("layer", layer).u("node", node).u("dest", key.first)
        .msg("steal a job from the most loaded node (" + std::to_string(victim) + ") to node " + std::to_string(node));
    load_[victim] = std::max<int64_t>(0, load_[victim] - 1);
    Job& j = jobs_[layer][key];
    j.sender = node;
    j.state = JobState::Sending;
    j.t_us = vclock::now_us();
    job_slots(node, key.first)++;
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
  // Every node takes its own jobs first, then steals: kicked one after
  // another, an early node would otherwise steal a later one's jobs before
  // that node had started any (e.g. a dest's load of its own copy).
  for (NodeID n : kick)
    while (assign_new_job(n, false)) {
    }
  for (NodeID n : kick)
    while (assign_new_job(n)) {
    }
}

}  // namespace dissem
