// Leader schedulers for modes 0 and 1 (reference: node.go:326-352 naive push,
// node.go:554-626 random-owner retransmit), with the planned data plane's
// relay broadcast, link-aware owners and relays around slow links.
#include "roles/node.h"

#include <algorithm>
#include <climits>
#include <set>
#include <tuple>

#include "core/log.h"
#include "core/trace.h"
#include "roles/node_internal.h"

namespace dissem {

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
    // Only ranks of the leader's own host can map its shared segment.
    if (cfg_.host_share && e_->planned())
      for (auto& st : status_) {
        if (host_of(st.first) != host_of(cfg_.id)) continue;
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

}  // namespace dissem
