// Several hosts (no reference counterpart: the reference's nodes are all
// peers on one network): per-host imports, relays inside a host over xGMI and
// the three-level mode-0 tree. Frozen scope: kept working under its tests
// (tests/test_multihost.py); the target is one 8-GPU node.
#include "roles/node.h"

#include <algorithm>
#include <climits>
#include <set>
#include <tuple>

#include "core/log.h"
#include "core/trace.h"
#include "roles/node_internal.h"

namespace dissem {

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

}  // namespace dissem
