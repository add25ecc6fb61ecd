// Leader-side failure handling (split out of node.cc): elastic recovery of
// the planned data plane (suspect -> probe -> shrink -> re-plan), mode-2 job
// retirement, host-engine job deadlines and re-dispatch, CRC NACKs.
#include <algorithm>
#include <climits>
#include <set>

#include "core/log.h"
#include "core/trace.h"
#include "roles/node.h"
#include "roles/node_internal.h"

namespace dissem {

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
  self_inflight_.clear();
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
    double dur = double(vclock::now_us() - job.t_us);
    auto& pf = perf_[job.sender];
    pf.first = pf.second == 0 ? dur : 0.5 * pf.first + 0.5 * dur;  // EWMA (quirk Q9)
    pf.second++;
    int& slots = job_slots(job.sender, key.first);
    slots = std::max(0, slots - 1);
    log::info(int64_t(cfg_.id)).u("node", job.sender).u("dest", key.first).u("layerID", layer).i("offset", key.second)
        .f("duration[ms]", dur / 1e3).msg("job completed");
  } else {
    load_[job.sender] = std::max<int64_t>(0, load_[job.sender] - 1);
  }
  while (assign_new_job(job.sender)) {
  }
}

// ------------------------------------------------------- failure handling

void Node::track(NodeID sender, NodeID dest, LayerID layer, int64_t off, int64_t size) {
  if (cfg_.job_timeout_s <= 0 || !is_leader_) return;
  outstanding_[{dest, layer}].push_back({sender, off, size, vclock::now_us()});
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
  const int64_t now = vclock::now_us();
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
          if (jt->second.state == JobState::Sending) {
            int& slots = job_slots(jt->second.sender, e.dest);
            slots = std::max(0, slots - 1);
          }
          jt->second.sender = alt;
          jt->second.state = JobState::Sending;
          jt->second.t_us = now;
          job_slots(alt, e.dest)++;
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
        while (assign_new_job(kv.first)) {
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

}  // namespace dissem
