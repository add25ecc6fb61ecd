// Leader-side job dispatch (split out of node.cc): transfer jobs with their
// chunk CRCs, the global sequence numbers of a transfer batch and its
// per-rank XferBatch messages, and the reference's retransmit request.
#include <algorithm>
#include <map>

#include "core/log.h"
#include "core/trace.h"
#include "roles/node.h"
#include "roles/node_internal.h"

namespace dissem {

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
  // sequence numbers spread over distinct xGMI links. This runs between
  // "timer start" and the first byte on any link: jobs are moved, not copied,
  // and the leader's own batch goes last (its engine starts staging the
  // moment it lands, beside the encoding of everyone else's).
  if (pending_jobs_.empty()) return;
  trace::Scoped tr("dissem.flush_batch");
  std::map<std::pair<int, std::pair<NodeID, NodeID>>, std::vector<size_t>> groups;  // (phase, (src, dst)) -> jobs
  for (size_t i = 0; i < pending_jobs_.size(); ++i)
    groups[{pending_jobs_[i].phase, {pending_jobs_[i].job.src, pending_jobs_[i].job.dst}}].push_back(i);
  std::map<NodeID, Message> per_rank;
  for (auto g = groups.begin(); g != groups.end();) {
    const int phase = g->first.first;
    auto end = g;
    while (end != groups.end() && end->first.first == phase) ++end;
    for (size_t round = 0;; ++round) {
      bool any = false;
      for (auto pr = g; pr != end; ++pr) {
        if (round >= pr->second.size()) continue;
        any = true;
        XferJob& j = pending_jobs_[pr->second[round]].job;
        j.seq = next_seq_++;
        if (j.dst == kAllRanks) {
          for (auto& st : status_)
            if (st.first != j.src) per_rank[st.first].jobs.push_back(j);
          per_rank[j.src].jobs.push_back(std::move(j));
        } else if (j.dst == j.src) {
          per_rank[j.src].jobs.push_back(std::move(j));
        } else {
          // a sender that announced the layer's manifest checks its staging
          // against its own CRCs: its copy of the job goes without them
          auto mh = manifest_holders_.find(j.layer);
          const bool own = mh != manifest_holders_.end() && mh->second.count(j.src);
          XferJob sj;
          sj.seq = j.seq;
          sj.src = j.src;
          sj.dst = j.dst;
          sj.layer = j.layer;
          sj.offset = j.offset;
          sj.size = j.size;
          sj.total = j.total;
          sj.chunk_bytes = j.chunk_bytes;
          sj.rate = j.rate;
          if (!own) sj.crc = j.crc;
          per_rank[j.src].jobs.push_back(std::move(sj));
          per_rank[j.dst].jobs.push_back(std::move(j));
        }
      }
      if (!any) break;
    }
    g = end;
  }
  pending_jobs_.clear();
  const uint64_t batch = next_batch_++;
  int64_t njobs = 0;
  std::vector<std::pair<NodeID, Message>> out;
  out.reserve(per_rank.size());
  for (auto& kv : per_rank)
    if (kv.first != cfg_.id) out.emplace_back(kv.first, std::move(kv.second));
  if (auto self = per_rank.find(cfg_.id); self != per_rank.end()) out.emplace_back(self->first, std::move(self->second));
  for (auto& o : out) {
    o.second.type = MsgType::XferBatch;
    o.second.batch = batch;
    o.second.order = cfg_.mode == 2 ? 1 : 0;  // pull jobs: job-major lanes (Message::order)
    o.second.src = cfg_.id;
    o.second.epoch = cfg_.epoch;
    njobs += int64_t(o.second.jobs.size());
  }
  try {
    t_->send_many(out);
  } catch (const std::exception& e) {
    log::error(int64_t(cfg_.id)).s("error", e.what()).msg("failed to send xfer_batch");
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

}  // namespace dissem
