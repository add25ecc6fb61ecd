// Planned engine (planned_engine.h), failure handling: stall reports to the
// leader (suspect peers), the communicator shrink around dead ranks, and the
// rank-death fault injection.
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

void PlannedEngine::die() {
  // Fault injection: this rank stops cold - no more posts, no acks, and its
  // control endpoint disappears (the leader's liveness probe sees it dead).
  log::warn(int64_t(self_node_)).i("groups", groups_issued_).msg("fault injection: rank dies");
  dead_ = true;
  backend_->crash();
  if (node_) node_->transport()->close();
}

std::vector<int> PlannedEngine::inflight_peers() const {
  std::vector<int> peers;
  for (auto& lane : inflight_)
    for (auto& g : lane)
      for (int p : g.peers)
        if (std::find(peers.begin(), peers.end(), p) == peers.end()) peers.push_back(p);
  return peers;
}

std::string PlannedEngine::describe_stall() const {
  // What each lane is waiting for (the stall report's detail): its in-flight
  // groups, the piece at the head of its queue and that chunk's state.
  std::string out;
  char buf[256];
  for (int l = 0; l < lanes_; ++l) {
    const auto& q = ops_[size_t(l)];
    if (q.empty() && inflight_[size_t(l)].empty()) continue;
    snprintf(buf, sizeof buf, "lane %d: %zu in flight, %zu queued", l, inflight_[size_t(l)].size(), q.size());
    out += buf;
    if (!q.empty()) {
      const Piece& p = q.front();
      auto it = layers_.find(p.layer);
      const int st = it != layers_.end() && p.chunk < int64_t(it->second.st.size()) ? it->second.st[size_t(p.chunk)] : -1;
      snprintf(buf, sizeof buf, "; head %s peer %d layer %llu chunk %lld key (%llu,%lld,%llu) chunk state %d",
               p.kind == Kind::Send ? "send" : "recv", p.peer, (unsigned long long)p.layer, (long long)p.chunk,
               (unsigned long long)p.batch, (long long)p.pidx, (unsigned long long)p.seq, st);
      out += buf;
    }
    out += " | ";
  }
  snprintf(buf, sizeof buf, "verifies %zu, disk: %zu waiting for a buffer, %d reading, %zu buffers free",
           verifies_.size(), disk_wait_.size(), disk_inflight_, bounce_free_.size());
  return out + buf;
}

void PlannedEngine::suspect(const std::vector<int>& peers, const std::string& why, bool broken) {
  if (broken && !recovering_) {
    recovering_ = true;  // the communicator is unusable until the Shrink
    recover_since_ = vclock::now();
  }
  Message m;
  m.type = MsgType::Suspect;
  for (int r : peers)
    if (r != cfg_.rank) m.peers.push_back(cfg_.rank_nodes[size_t(r)]);
  log::warn(int64_t(self_node_)).s("why", why).i("peers", int64_t(m.peers.size())).s("state", describe_stall())
      .msg("data plane stalled: reporting suspect peers to the leader");
  trace::mark("dissem.suspect");
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.suspects++;
  }
  if (node_) node_->send_msg(node_->leader(), m);
}

void PlannedEngine::do_shrink(const std::vector<NodeID>& dead_nodes, uint64_t generation,
                              const std::string& comm_id) {
  // Every survivor runs this for the same generation: abort what is in flight,
  // continue on a communicator without the dead ranks, forget every chunk that
  // was not verified resident (the leader re-plans whole layers that were not acked).
  trace::Scoped tr("dissem.shrink");
  std::vector<int> dead;
  for (NodeID n : dead_nodes) {
    auto it = node_rank_.find(n);
    if (it != node_rank_.end()) dead.push_back(it->second);
  }
  std::sort(dead.begin(), dead.end());
  const int old_rank = cfg_.rank;
  int64_t aborted = 0;
  for (auto& q : ops_) aborted += int64_t(q.size());
  int new_rank;
  {
    CallMark cm(this, "shrink", -1);
    new_rank = backend_->shrink(dead, generation, comm_id);
  }
  for (auto& lane : inflight_) {
    for (auto& g : lane) backend_->release(g.ev);
    lane.clear();
  }
  for (auto& v : verifies_) {
    aborted += int64_t(v.pieces.size());
    backend_->release(v.ev);
  }
  verifies_.clear();
  aborted += int64_t(pending_checks_.size());
  drop_pending_checks();
  for (auto& b : bounce_busy_) {  // every queue drained in the backend's shrink: the copies are done
    ev_drop(b.first);
    bounce_free_.push_back(b.second);
  }
  bounce_busy_.clear();
  for (auto& q : ops_) q.clear();
  restage_.clear();
  local_wait_.clear();
  deferred_local_.clear();
  promoting_.clear();
  fwd_pending_.clear();
  for (auto& kv : layers_) {
    Layer& L = kv.second;
    for (size_t c = 0; c < L.st.size(); ++c) {
      if (L.st[c] == 1 || L.st[c] == 4) L.st[c] = 0;  // pending or bad: gone (st 3: its disk read still lands)
      set_chunk_ev(L, int64_t(c), 0);
      L.fails[c] = 0;
    }
    L.part.clear();
  }
  std::vector<NodeID> nodes;
  for (int r = 0; r < cfg_.world; ++r)
    if (!std::binary_search(dead.begin(), dead.end(), r)) nodes.push_back(cfg_.rank_nodes[size_t(r)]);
  cfg_.rank_nodes = nodes;
  cfg_.world = int(nodes.size());
  cfg_.hosts = 1;  // the survivors no longer fill whole hosts: per-distance lanes (as the backend's)
  cfg_.rank = new_rank;
  node_rank_.clear();
  for (int r = 0; r < cfg_.world; ++r) node_rank_[cfg_.rank_nodes[size_t(r)]] = r;
  recovering_ = false;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);
    stats_.shrinks++;
    stats_.aborted_pieces += aborted;
    stats_.comm_reform_ms = backend_->comm_init_ms();  // the survivors' communicators, set up like the first
  }
  log::warn(int64_t(self_node_)).i("dead", int64_t(dead.size())).i("old_rank", old_rank).i("new_rank", new_rank)
      .i("world", cfg_.world).i("aborted_pieces", aborted).msg("communicator shrunk: continuing without dead ranks");
  if (node_) {
    // Through the node's inbox, so acks for chunks that landed before the
    // shrink reach the leader first.
    auto d = std::make_shared<Message>();
    d->type = MsgType::ShrinkDone;
    d->seq = generation;
    d->src = self_node_;
    d->epoch = node_->epoch();
    node_->inject(d);
  }
}

}  // namespace dissem
