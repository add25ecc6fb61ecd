#include "sched/maxflow.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <queue>
#include <set>
#include <tuple>

#include "core/trace.h"

namespace dissem {

namespace {

constexpr int64_t kInf = int64_t(4e18);

struct Dinic {
  struct E {
    int to;
    int64_t cap;
  };
  std::vector<E> e;
  std::vector<std::vector<int>> g;
  std::vector<int> level, it;
  explicit Dinic(int n) : g(size_t(n)), level(size_t(n)), it(size_t(n)) {}
  int add(int u, int v, int64_t c) {
    e.push_back({v, c});
    g[size_t(u)].push_back(int(e.size()) - 1);
    e.push_back({u, 0});
    g[size_t(v)].push_back(int(e.size()) - 1);
    return int(e.size()) - 2;
  }
  bool bfs(int s, int t) {
    std::fill(level.begin(), level.end(), -1);
    std::queue<int> q;
    level[size_t(s)] = 0;
    q.push(s);
    while (!q.empty()) {
      int u = q.front();
      q.pop();
      for (int id : g[size_t(u)])
        if (e[size_t(id)].cap > 0 && level[size_t(e[size_t(id)].to)] < 0) {
          level[size_t(e[size_t(id)].to)] = level[size_t(u)] + 1;
          q.push(e[size_t(id)].to);
        }
    }
    return level[size_t(t)] >= 0;
  }
  int64_t dfs(int u, int t, int64_t f) {
    if (u == t) return f;
    for (int& i = it[size_t(u)]; i < int(g[size_t(u)].size()); ++i) {
      int id = g[size_t(u)][size_t(i)];
      E& ed = e[size_t(id)];
      if (ed.cap > 0 && level[size_t(ed.to)] == level[size_t(u)] + 1) {
        int64_t d = dfs(ed.to, t, std::min(f, ed.cap));
        if (d > 0) {
          ed.cap -= d;
          e[size_t(id ^ 1)].cap += d;
          return d;
        }
      }
    }
    return 0;
  }
  int64_t run(int s, int t) {
    int64_t flow = 0;
    while (bfs(s, t)) {
      std::fill(it.begin(), it.end(), 0);
      while (int64_t f = dfs(s, t, kInf)) {
        flow += f;
        if (flow >= kInf) return flow;
      }
    }
    return flow;
  }
  int64_t flow_on(int id) const { return e[size_t(id ^ 1)].cap; }
};

int64_t cap_for(int64_t rate_bps, double T) {
  if (rate_bps <= 0) return kInf;
  double c = double(rate_bps) * T;
  if (c >= 4e18) return kInf;
  return int64_t(std::floor(c));
}

struct Built {
  std::unique_ptr<Dinic> d;
  int src = 0, sink = 1;
  // (sender, layer, dest) -> edge id carrying its bytes
  std::map<std::tuple<NodeID, LayerID, NodeID>, int> job_edges;
};

Built build(const FlowProblem& p, double T) {
  // demands indexed by layer
  std::map<LayerID, std::vector<const FlowDemand*>> by_layer;
  for (auto& dm : p.demands) by_layer[dm.layer].push_back(&dm);
  std::map<std::pair<LayerID, NodeID>, int64_t> dsize;
  for (auto& dm : p.demands) dsize[{dm.layer, dm.dest}] = std::max(dsize[{dm.layer, dm.dest}], dm.size);
  const bool topo = !p.link_bps.empty();
  const int kDevice = int(SourceType::Device);
  // Candidate (sender, tier, layer, dest) edges, and per (sender, dest) the
  // demanded bytes by tier (to split a link shared by several tiers).
  struct Cand {
    NodeID s;
    int t;
    LayerID l;
    NodeID d;
  };
  std::vector<Cand> cands;
  std::map<std::pair<NodeID, NodeID>, std::map<int, int64_t>> sd_tiers;
  std::set<std::tuple<NodeID, LayerID, NodeID>> seen;
  for (auto& hs : p.holdings) {
    const NodeID s = hs.first;
    for (auto& lm : hs.second) {
      auto bl = by_layer.find(lm.first);
      if (bl == by_layer.end()) continue;
      const int t = int(lm.second.source_type);
      for (auto* dm : bl->second) {
        if (dm->dest == s && !p.allow_self) continue;
        if (!seen.insert({s, lm.first, dm->dest}).second) continue;
        cands.push_back({s, t, lm.first, dm->dest});
        sd_tiers[{s, dm->dest}][t] += dsize[{lm.first, dm->dest}];
      }
    }
  }
  // Vertex numbering: 0 source, 1 sink.
  int n = 2;
  std::map<NodeID, int> vs, vstage, vdest;
  std::map<std::pair<NodeID, int>, int> vst;
  std::map<std::tuple<NodeID, int, NodeID>, int> vlink;  // (s, tier or -1 = shared, d)
  std::map<std::pair<LayerID, NodeID>, int> vd;
  for (auto& kv : dsize) {
    vd[kv.first] = n++;
    if (!vdest.count(kv.first.second)) vdest[kv.first.second] = n++;
  }
  auto link_key = [&](const Cand& c) {
    return std::make_tuple(c.s, sd_tiers[{c.s, c.d}].size() > 1 ? c.t : -1, c.d);
  };
  for (auto& c : cands) {
    if (!vs.count(c.s)) vs[c.s] = n++;
    if (c.t != kDevice && !vstage.count(c.s)) vstage[c.s] = n++;
    if (!vst.count({c.s, c.t})) vst[{c.s, c.t}] = n++;
    if (topo && c.s != c.d && !vlink.count(link_key(c))) vlink[link_key(c)] = n++;
  }
  Built b;
  b.d = std::make_unique<Dinic>(n);
  Dinic& d = *b.d;
  auto rate_of = [](const std::map<NodeID, int64_t>& m, NodeID k) {
    auto it = m.find(k);
    return it == m.end() ? int64_t(0) : it->second;
  };
  for (auto& kv : vs) d.add(b.src, kv.second, cap_for(rate_of(p.egress_bps, kv.first), T));
  // Staging is paid once per byte a sender loads into HBM, however many dests it
  // then forwards it to over xGMI; a flow charges every transfer, so the
  // budget is scaled by the sender's fan-out (its candidate bytes over the
  // distinct layer bytes it could load) - exact when its layers share one
  // fan-out.
  std::map<NodeID, double> cand_bytes, layer_bytes;
  std::set<std::pair<NodeID, LayerID>> counted;
  for (auto& c : cands) {
    if (c.t == kDevice) continue;
    cand_bytes[c.s] += double(dsize[{c.l, c.d}]);
    if (counted.insert({c.s, c.l}).second) {
      int64_t mx = 0;
      for (auto* dm : by_layer[c.l]) mx = std::max(mx, dm->size);
      layer_bytes[c.s] += double(mx);
    }
  }
  for (auto& kv : vstage) {
    const int64_t r = rate_of(p.stage_bps, kv.first);
    const double fan = layer_bytes[kv.first] > 0 ? std::max(1.0, cand_bytes[kv.first] / layer_bytes[kv.first]) : 1.0;
    d.add(vs[kv.first], kv.second, r > 0 ? cap_for(int64_t(double(r) * fan), T) : kInf);
  }
  // Tier capacity: the tier's configured rate (all its layers share one device).
  std::map<std::pair<NodeID, int>, int64_t> tier_rate;
  for (auto& hs : p.holdings)
    for (auto& lm : hs.second) {
      auto key = std::make_pair(hs.first, int(lm.second.source_type));
      if (!vst.count(key)) continue;
      int64_t r = lm.second.limit_rate;
      auto it = tier_rate.find(key);
      if (it == tier_rate.end()) tier_rate[key] = r;
      else if (it->second > 0 && (r <= 0 || r > it->second)) it->second = r;  // 0 = unlimited wins
    }
  for (auto& kv : vst) {
    const NodeID s = kv.first.first;
    const int parent = kv.first.second == kDevice ? vs[s] : vstage[s];
    d.add(parent, kv.second, cap_for(tier_rate[kv.first], T));
  }
  for (auto& kv : vlink) {
    const NodeID s = std::get<0>(kv.first), dst = std::get<2>(kv.first);
    const int t = std::get<1>(kv.first);
    auto lk = p.link_bps.find({s, dst});
    int64_t cap = cap_for(lk == p.link_bps.end() ? 0 : lk->second, T);
    const auto& tiers = sd_tiers[{s, dst}];
    if (t >= 0 && cap < kInf) {
      // several tiers share this link: each gets its share of the demanded bytes
      int64_t tot = 0;
      for (auto& x : tiers) tot += x.second;
      cap = tot > 0 ? int64_t(double(cap) * double(tiers.at(t)) / double(tot)) : cap;
    }
    // a shared vertex is fed by every tier of the sender that serves this dest
    if (t >= 0) {
      d.add(vst[{s, t}], kv.second, cap);
    } else {
      const int only = tiers.begin()->first;
      d.add(vst[{s, only}], kv.second, cap);
    }
  }
  for (auto& c : cands) {
    auto key = std::make_tuple(c.s, c.l, c.d);
    const int from = (topo && c.s != c.d) ? vlink[link_key(c)] : vst[{c.s, c.t}];
    b.job_edges[key] = d.add(from, vd[{c.l, c.d}], kInf);
  }
  for (auto& kv : vd) d.add(kv.second, vdest[kv.first.second], dsize[kv.first]);
  for (auto& kv : vdest) d.add(kv.second, b.sink, cap_for(rate_of(p.ingress_bps, kv.first), T));
  return b;
}

int64_t required_bytes(const FlowProblem& p) {
  std::map<std::pair<LayerID, NodeID>, int64_t> dsize;
  for (auto& dm : p.demands) dsize[{dm.layer, dm.dest}] = std::max(dsize[{dm.layer, dm.dest}], dm.size);
  int64_t r = 0;
  for (auto& kv : dsize) r += kv.second;
  return r;
}

}  // namespace

int64_t max_flow_at(const FlowProblem& p, double T) {
  Built b = build(p, T);
  return b.d->run(b.src, b.sink);
}

FlowPlan solve_flow(const FlowProblem& p) {
  trace::Scoped tr("dissem.maxflow");
  FlowPlan plan;
  plan.required = required_bytes(p);
  if (plan.required == 0) {
    plan.feasible = true;
    return plan;
  }
  auto flow = [&](double T) {
    ++plan.solves;
    return max_flow_at(p, T);
  };
  // Upper bound by doubling (flow.go:155-167).
  double hi = p.integer_seconds ? 1.0 : 1e-3;
  bool found = false;
  for (int i = 0; i < 128; ++i) {
    if (flow(hi) >= plan.required) {
      found = true;
      break;
    }
    hi *= 2;
  }
  if (!found) return plan;  // infeasible (some demand has no holder)
  double T = hi;
  if (p.integer_seconds) {
    // Bisection over integers in [1, hi] (flow.go:171-187).
    int64_t l = 1, r = int64_t(hi), best = int64_t(hi);
    while (l <= r) {
      int64_t m = l + (r - l) / 2;
      if (flow(double(m)) < plan.required) {
        l = m + 1;
      } else {
        best = std::min(best, m);
        r = m - 1;
      }
    }
    T = double(best);
  } else {
    double lo = hi / 2;
    if (lo < 1e-9 || flow(lo) >= plan.required) lo = 0;
    for (int i = 0; i < 60 && (hi - lo) > hi * 1e-6; ++i) {
      double m = 0.5 * (lo + hi);
      if (flow(m) >= plan.required) hi = m;
      else lo = m;
    }
    T = hi;
  }
  // Re-solve at T and read the per-(sender, layer, dest) flows.
  Built b = build(p, T);
  ++plan.solves;
  plan.max_flow = b.d->run(b.src, b.sink);
  plan.T = T;
  plan.feasible = plan.max_flow >= plan.required;
  std::map<std::pair<LayerID, NodeID>, std::vector<FlowJob>> per_demand;
  for (auto& kv : b.job_edges) {
    int64_t f = b.d->flow_on(kv.second);
    if (f <= 0) continue;
    per_demand[{std::get<1>(kv.first), std::get<2>(kv.first)}].push_back(
        FlowJob{std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first), f, 0});
  }
  for (auto& kv : per_demand) {
    auto& jobs = kv.second;
    if (p.align > 1 && jobs.size() > 1) {
      int64_t total = 0;
      for (auto& j : jobs) total += j.size;
      int64_t acc = 0;
      size_t biggest = 0;
      for (size_t i = 0; i < jobs.size(); ++i) {
        jobs[i].size = (jobs[i].size / p.align) * p.align;
        acc += jobs[i].size;
        if (jobs[i].size > jobs[biggest].size) biggest = i;
      }
      jobs[biggest].size += total - acc;
      jobs.erase(std::remove_if(jobs.begin(), jobs.end(), [](const FlowJob& j) { return j.size <= 0; }),
                 jobs.end());
    }
    int64_t off = 0;  // ranges partition the layer, senders in id order
    for (auto& j : jobs) {
      j.offset = off;
      off += j.size;
      plan.jobs.push_back(j);
    }
  }
  return plan;
}

}  // namespace dissem
