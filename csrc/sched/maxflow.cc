#include "sched/maxflow.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <queue>
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
  // Vertex numbering.
  std::map<NodeID, int> vs;
  std::map<std::pair<NodeID, int>, int> vst;
  std::map<std::tuple<NodeID, int, NodeID>, int> vlink;
  std::map<std::pair<LayerID, NodeID>, int> vd;
  std::map<NodeID, int> vdest;
  int n = 2;
  // demands indexed by layer
  std::map<LayerID, std::vector<const FlowDemand*>> by_layer;
  for (auto& dm : p.demands) {
    by_layer[dm.layer].push_back(&dm);
    if (!vd.count({dm.layer, dm.dest})) vd[{dm.layer, dm.dest}] = n++;
    if (!vdest.count(dm.dest)) vdest[dm.dest] = n++;
  }
  const bool topo = !p.link_bps.empty();
  for (auto& hs : p.holdings) {
    NodeID s = hs.first;
    for (auto& lm : hs.second) {
      auto bl = by_layer.find(lm.first);
      if (bl == by_layer.end()) continue;
      int t = int(lm.second.source_type);
      for (auto* dm : bl->second) {
        if (dm->dest == s && !p.allow_self) continue;
        if (!vs.count(s)) vs[s] = n++;
        if (!vst.count({s, t})) vst[{s, t}] = n++;
        if (topo && !vlink.count({s, t, dm->dest})) vlink[{s, t, dm->dest}] = n++;
      }
    }
  }
  Built b;
  b.d = std::make_unique<Dinic>(n);
  Dinic& d = *b.d;
  for (auto& kv : vs) {
    auto eg = p.egress_bps.find(kv.first);
    d.add(b.src, kv.second, cap_for(eg == p.egress_bps.end() ? 0 : eg->second, T));
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
  for (auto& kv : vst) d.add(vs[kv.first.first], kv.second, cap_for(tier_rate[kv.first], T));
  for (auto& kv : vlink) {
    NodeID s = std::get<0>(kv.first), dst = std::get<2>(kv.first);
    auto lk = p.link_bps.find({s, dst});
    int64_t rate = lk == p.link_bps.end() ? 0 : lk->second;
    if (s == dst) rate = 0;  // a self-load does not use a network link
    d.add(vst[{s, std::get<1>(kv.first)}], kv.second, cap_for(rate, T));
  }
  for (auto& hs : p.holdings) {
    NodeID s = hs.first;
    for (auto& lm : hs.second) {
      auto bl = by_layer.find(lm.first);
      if (bl == by_layer.end()) continue;
      int t = int(lm.second.source_type);
      for (auto* dm : bl->second) {
        if (dm->dest == s && !p.allow_self) continue;
        auto key = std::make_tuple(s, lm.first, dm->dest);
        if (b.job_edges.count(key)) continue;
        int from = topo ? vlink[{s, t, dm->dest}] : vst[{s, t}];
        b.job_edges[key] = d.add(from, vd[{dm->layer, dm->dest}], kInf);
      }
    }
  }
  std::map<std::pair<LayerID, NodeID>, int64_t> dsize;
  for (auto& dm : p.demands) dsize[{dm.layer, dm.dest}] = std::max(dsize[{dm.layer, dm.dest}], dm.size);
  for (auto& kv : vd) d.add(kv.second, vdest[kv.first.second], dsize[kv.first]);
  for (auto& kv : vdest) {
    auto in = p.ingress_bps.find(kv.first);
    d.add(kv.second, b.sink, cap_for(in == p.ingress_bps.end() ? 0 : in->second, T));
  }
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
