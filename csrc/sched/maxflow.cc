#include "sched/maxflow.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <queue>
#include <set>
#include <tuple>

#include "core/trace.h"
#include "sched/lp.h"

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
    const bool dev = kv.first.second == kDevice;
    const int parent = dev ? vs[s] : vstage[s];
    int64_t r = tier_rate[kv.first];
    if (p.stage_once && !dev && r > 0 && layer_bytes[s] > 0)  // read once, forwarded to every dest
      r = int64_t(double(r) * std::max(1.0, cand_bytes[s] / layer_bytes[s]));
    d.add(parent, kv.second, cap_for(r, T));
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

// Layers with the same holders (and tiers) and the same demands (dest, bytes):
// one LP class. Its demand per dest is the sum over its layers, and an LP
// solution splits back onto the layers in equal shares - exact, as every
// layer of a class has the same constraints.
struct LpClass {
  std::vector<std::pair<NodeID, int>> holders;   // (sender, tier)
  std::vector<std::pair<NodeID, int64_t>> dests; // (dest, bytes per layer)
  std::vector<std::pair<NodeID, int64_t>> self;  // holders that load it for themselves (bytes per layer)
  std::vector<LayerID> layers;
};

std::vector<LpClass> lp_classes(const FlowProblem& p) {
  std::map<LayerID, std::vector<std::pair<NodeID, int>>> holders;
  for (auto& hs : p.holdings)
    for (auto& lm : hs.second) holders[lm.first].push_back({hs.first, int(lm.second.source_type)});
  std::map<LayerID, std::map<NodeID, int64_t>> dem;  // layer -> dest -> bytes
  for (auto& dm : p.demands) {
    int64_t& z = dem[dm.layer][dm.dest];
    z = std::max(z, dm.size);
  }
  std::map<LayerID, std::map<NodeID, int64_t>> selfl;  // layer -> loading holder -> bytes
  for (auto& kv : p.self_loads)
    for (auto& ls : kv.second) selfl[ls.first][kv.first] = ls.second;
  using Key = std::tuple<std::vector<std::pair<NodeID, int>>, std::vector<std::pair<NodeID, int64_t>>,
                         std::vector<std::pair<NodeID, int64_t>>>;
  std::map<Key, size_t> index;
  std::vector<LpClass> out;
  for (auto& kv : selfl) dem[kv.first];  // a layer only its holders load still draws on their budgets
  for (auto& kv : dem) {
    auto h = holders[kv.first];
    std::sort(h.begin(), h.end());
    std::vector<std::pair<NodeID, int64_t>> ds(kv.second.begin(), kv.second.end());
    std::vector<std::pair<NodeID, int64_t>> sl;
    if (auto it = selfl.find(kv.first); it != selfl.end()) sl.assign(it->second.begin(), it->second.end());
    Key key{h, ds, sl};
    auto it = index.find(key);
    if (it == index.end()) {
      it = index.emplace(key, out.size()).first;
      out.push_back(LpClass{h, ds, sl, {}});
    }
    out[it->second].layers.push_back(kv.first);
  }
  return out;
}

// Byte counts per (sender, layer, dest) -> ranges: per demand, aligned sizes
// (remainder to the biggest), offsets in sender order, so a sender that serves
// one layer to several dests sends each of them the same region where it can.
void extract_jobs(std::map<std::pair<LayerID, NodeID>, std::vector<FlowJob>>& per_demand, int64_t align,
                  FlowPlan& plan) {
  for (auto& kv : per_demand) {
    auto& jobs = kv.second;
    if (align > 1 && jobs.size() > 1) {
      int64_t total = 0;
      for (auto& j : jobs) total += j.size;
      int64_t acc = 0;
      size_t biggest = 0;
      for (size_t i = 0; i < jobs.size(); ++i) {
        jobs[i].size = (jobs[i].size / align) * align;
        acc += jobs[i].size;
        if (jobs[i].size > jobs[biggest].size) biggest = i;
      }
      jobs[biggest].size += total - acc;
      jobs.erase(std::remove_if(jobs.begin(), jobs.end(), [](const FlowJob& j) { return j.size <= 0; }), jobs.end());
    }
    int64_t off = 0;  // ranges partition the layer, senders in id order
    for (auto& j : jobs) {
      j.offset = off;
      off += j.size;
      plan.jobs.push_back(j);
    }
  }
}

FlowPlan solve_flow_lp(const FlowProblem& p) {
  trace::Scoped tr("dissem.plan_lp");
  FlowPlan plan;
  plan.solver = "lp";
  plan.required = required_bytes(p);
  const int kDevice = int(SourceType::Device), kDisk = int(SourceType::Disk);
  const auto classes = lp_classes(p);
  // Scale: bytes by the largest class, rates by the largest rate -> O(1) coefficients.
  double B0 = 1, R0 = 1;
  for (auto& c : classes)
    for (auto& d : c.dests) B0 = std::max(B0, double(d.second) * double(c.layers.size()));
  auto upd = [&](int64_t r) {
    if (r > 0) R0 = std::max(R0, double(r));
  };
  for (auto& kv : p.egress_bps) upd(kv.second);
  for (auto& kv : p.ingress_bps) upd(kv.second);
  for (auto& kv : p.link_bps) upd(kv.second);
  for (auto& kv : p.stage_bps) upd(kv.second);
  for (auto& kv : p.disk_group_bps) upd(kv.second);
  for (auto& kv : p.nic_bps) upd(kv.second);
  for (auto& hs : p.holdings)
    for (auto& lm : hs.second) upd(lm.second.limit_rate);
  LpProblem lp;
  lp.n = 1;  // column 0 = T (scaled)
  struct X {
    size_t c;
    NodeID s;
    int t;
    NodeID d;
    int col;
  };
  std::vector<X> xs;
  std::map<std::pair<size_t, NodeID>, int> ycol;  // (class, sender) -> y column
  for (size_t ci = 0; ci < classes.size(); ++ci) {
    const LpClass& c = classes[ci];
    for (auto& dz : c.dests) {
      const NodeID d = dz.first;
      LpRow dem;
      dem.b = double(dz.second) * double(c.layers.size()) / B0;
      for (auto& h : c.holders) {
        if (h.first == d && !p.allow_self) continue;
        xs.push_back(X{ci, h.first, h.second, d, lp.n});
        dem.a.push_back({lp.n++, 1.0});
      }
      if (dem.a.empty()) return plan;  // a demand nobody can serve
      lp.eq.push_back(dem);
    }
    // y = bytes of the class a sender loads into HBM (staged once, forwarded to
    // every dest): the staging budget always charges y; tier rates and disk
    // groups charge it with stage_once, else every transfer re-reads.
    for (auto& h : c.holders) {
      auto st = p.stage_bps.find(h.first);
      if (h.second != kDevice && (p.stage_once || (st != p.stage_bps.end() && st->second > 0)))
        ycol[{ci, h.first}] = lp.n++;
    }
    // A holder that also loads the layer for itself loads all of it: y >= its bytes
    // (as an equality with a surplus column: y - surplus = bytes).
    for (auto& sl : c.self) {
      auto y = ycol.find({ci, sl.first});
      if (y == ycol.end()) continue;
      LpRow r;
      r.a = {{y->second, 1.0}, {lp.n++, -1.0}};
      r.b = double(sl.second) * double(c.layers.size()) / B0;
      lp.eq.push_back(r);
    }
  }
  lp.c.assign(size_t(lp.n), 0.0);
  lp.c[0] = 1.0;
  // x - y <= 0: what a sender forwards of a class to any one dest it must have loaded
  for (size_t i = 0; i < xs.size(); ++i) {
    auto y = ycol.find({xs[i].c, xs[i].s});
    if (y == ycol.end()) continue;
    LpRow r;
    r.a = {{xs[i].col, 1.0}, {y->second, -1.0}};
    lp.le.push_back(r);
  }
  auto budget = [&](int64_t rate, const std::vector<std::pair<int, double>>& cols) {
    if (rate <= 0 || cols.empty()) return;
    LpRow r;
    std::map<int, double> merged;
    for (auto& e : cols) merged[e.first] += e.second;
    for (auto& e : merged) r.a.push_back(e);
    r.a.push_back({0, -double(rate)});  // scaled by the candidate R0 below
    lp.le.push_back(r);
  };
  auto rate_of = [](const std::map<NodeID, int64_t>& m, NodeID k) {
    auto it = m.find(k);
    return it == m.end() ? int64_t(0) : it->second;
  };
  std::map<NodeID, std::vector<std::pair<int, double>>> egress, ingress, stage, nic_out, nic_in;
  auto host_of = [&](NodeID n) {
    auto it = p.host.find(n);
    return it == p.host.end() ? 0 : it->second;
  };
  std::map<std::pair<NodeID, NodeID>, std::vector<std::pair<int, double>>> link;
  std::map<std::pair<NodeID, int>, std::vector<std::pair<int, double>>> tier;
  std::map<int, std::vector<std::pair<int, double>>> group;
  for (size_t i = 0; i < xs.size(); ++i) {
    const X& x = xs[i];
    const int col = x.col;
    egress[x.s].push_back({col, 1.0});
    ingress[x.d].push_back({col, 1.0});
    if (x.s != x.d) link[{x.s, x.d}].push_back({col, 1.0});
    if (host_of(x.s) != host_of(x.d)) {
      nic_out[x.s].push_back({col, 1.0});
      nic_in[x.d].push_back({col, 1.0});
    }
    const bool y = ycol.count({x.c, x.s}) > 0;
    if (!y || !p.stage_once) {  // read per transfer
      tier[{x.s, x.t}].push_back({col, 1.0});
      auto g = p.disk_group.find(x.s);
      if (x.t == kDisk && g != p.disk_group.end()) group[g->second].push_back({col, 1.0});
    }
    if (!y && x.t != kDevice) stage[x.s].push_back({col, 1.0});
  }
  for (auto& kv : ycol) {
    const size_t ci = kv.first.first;
    const NodeID s = kv.first.second;
    int t = kDevice;
    for (auto& h : classes[ci].holders)
      if (h.first == s) t = h.second;
    stage[s].push_back({kv.second, 1.0});
    if (p.stage_once) {  // read once
      tier[{s, t}].push_back({kv.second, 1.0});
      auto g = p.disk_group.find(s);
      if (t == kDisk && g != p.disk_group.end()) group[g->second].push_back({kv.second, 1.0});
    }
  }
  for (auto& kv : egress) budget(rate_of(p.egress_bps, kv.first), kv.second);
  for (auto& kv : ingress) budget(rate_of(p.ingress_bps, kv.first), kv.second);
  for (auto& kv : stage) budget(rate_of(p.stage_bps, kv.first), kv.second);
  for (auto& kv : nic_out) budget(rate_of(p.nic_bps, kv.first), kv.second);
  for (auto& kv : nic_in) budget(rate_of(p.nic_bps, kv.first), kv.second);
  for (auto& kv : link) {
    auto it = p.link_bps.find(kv.first);
    if (it != p.link_bps.end()) budget(it->second, kv.second);
  }
  // tier rate: the tier's configured rate (its layers share one device; 0 = unlimited wins)
  std::map<std::pair<NodeID, int>, int64_t> tier_rate;
  for (auto& hs : p.holdings)
    for (auto& lm : hs.second) {
      auto key = std::make_pair(hs.first, int(lm.second.source_type));
      const int64_t r = lm.second.limit_rate;
      auto it = tier_rate.find(key);
      if (it == tier_rate.end()) tier_rate[key] = r;
      else if (it->second > 0 && (r <= 0 || r > it->second)) it->second = r;
    }
  for (auto& kv : tier) budget(tier_rate[kv.first], kv.second);
  for (auto& kv : group) {
    auto it = p.disk_group_bps.find(kv.first);
    if (it != p.disk_group_bps.end()) budget(it->second, kv.second);
  }
  // T's column carries -rate / R0. R0 = the largest rate keeps every
  // coefficient <= 1, but when the rates span orders of magnitude (measured
  // link rates next to planning constants) the optimum's scaled T grows large
  // and the dense simplex can lose it to round-off (it has reported such
  // instances "unbounded"/"infeasible" where scipy finds the optimum): retry
  // with the median and the smallest rate as the scale.
  std::vector<double> rates;
  for (auto& row : lp.le)
    for (auto& e : row.a)
      if (e.first == 0 && e.second < 0) rates.push_back(-e.second);
  std::sort(rates.begin(), rates.end());
  std::vector<double> scales{R0};
  if (!rates.empty()) {
    scales.push_back(rates[rates.size() / 2]);
    scales.push_back(rates.front());
  }
  LpResult r;
  LpProblem scaled;
  for (double sc : scales) {
    scaled = lp;
    for (auto& row : scaled.le)
      for (auto& e : row.a)
        if (e.first == 0) e.second /= sc;
    r = solve_lp(scaled);
    plan.lp_pivots += r.pivots;
    if (r.ok) {
      R0 = sc;
      break;
    }
  }
  if (getenv("DLD_LP_DUMP")) {
    const LpProblem& lp = scaled;
    fprintf(stderr, "LP n=%d B0=%g R0=%g\n", lp.n, B0, R0);
    for (auto& row : lp.eq) {
      fprintf(stderr, "EQ");
      for (auto& e : row.a) fprintf(stderr, " %d:%g", e.first, e.second);
      fprintf(stderr, " = %g\n", row.b);
    }
    for (auto& row : lp.le) {
      fprintf(stderr, "LE");
      for (auto& e : row.a) fprintf(stderr, " %d:%g", e.first, e.second);
      fprintf(stderr, " <= %g\n", row.b);
    }
    fprintf(stderr, "status %s obj %g\n", r.status.c_str(), r.obj);
  }
  plan.lp_status = r.status;
  if (!r.ok) return plan;
  double T = r.x[0] * B0 / R0;
  if (p.integer_seconds) T = std::max(1.0, std::ceil(T - 1e-9));
  plan.T = T;
  plan.max_flow = plan.required;
  plan.feasible = true;
  plan.solves = 1;
  // Class bytes back to layers (each layer of a class takes its share of every x).
  std::map<std::pair<LayerID, NodeID>, std::vector<FlowJob>> per_demand;
  for (size_t i = 0; i < xs.size(); ++i) {
    const double bytes = r.x[size_t(xs[i].col)] * B0;
    if (bytes <= 0.5) continue;
    const LpClass& c = classes[xs[i].c];
    for (LayerID l : c.layers)
      per_demand[{l, xs[i].d}].push_back(FlowJob{xs[i].s, l, xs[i].d, int64_t(bytes / double(c.layers.size())), 0});
  }
  // Integer bytes: every demand's shares add up to its size exactly (remainder to the biggest share).
  std::map<std::pair<LayerID, NodeID>, int64_t> dsize;
  for (auto& dm : p.demands) dsize[{dm.layer, dm.dest}] = std::max(dsize[{dm.layer, dm.dest}], dm.size);
  for (auto& kv : per_demand) {
    auto& jobs = kv.second;
    std::sort(jobs.begin(), jobs.end(), [](const FlowJob& a, const FlowJob& b) { return a.sender < b.sender; });
    int64_t acc = 0;
    size_t biggest = 0;
    for (size_t i = 0; i < jobs.size(); ++i) {
      acc += jobs[i].size;
      if (jobs[i].size > jobs[biggest].size) biggest = i;
    }
    jobs[biggest].size += dsize[kv.first] - acc;
  }
  extract_jobs(per_demand, p.align, plan);
  return plan;
}

}  // namespace

bool needs_lp(const FlowProblem& p) {
  if (p.solver == "lp") return true;
  if (p.solver == "flow") return false;
  const int kDevice = int(SourceType::Device), kDisk = int(SourceType::Disk);
  // a NIC shared by a node's traffic to every other host: the LP's rows
  {
    std::set<int> hosts;
    for (auto& kv : p.host) hosts.insert(kv.second);
    if (hosts.size() > 1)
      for (auto& kv : p.nic_bps)
        if (kv.second > 0) return true;
  }
  std::map<LayerID, std::map<NodeID, int64_t>> dests;  // layer -> dest -> bytes
  for (auto& dm : p.demands) {
    int64_t& z = dests[dm.layer][dm.dest];
    z = std::max(z, dm.size);
  }
  std::map<std::pair<NodeID, NodeID>, std::set<int>> sd_tiers;
  std::map<NodeID, std::set<double>> fanouts;  // effective fan-out: bytes sent per byte loaded
  std::map<NodeID, bool> tier_capped;  // a non-HBM tier with a finite rate
  for (auto& hs : p.holdings)
    for (auto& lm : hs.second) {
      auto it = dests.find(lm.first);
      if (it == dests.end()) continue;
      const int t = int(lm.second.source_type);
      int64_t sent = 0, loaded = 0;
      for (auto& dz : it->second) {
        if (dz.first == hs.first && !p.allow_self) continue;
        sd_tiers[{hs.first, dz.first}].insert(t);
        sent += dz.second;
        loaded = std::max(loaded, dz.second);
      }
      if (loaded == 0) continue;
      const double fan = std::round(double(sent) / double(loaded) * 1e9) / 1e9;
      // a disk shared with other senders
      if (t == kDisk && p.disk_group.count(hs.first) && p.disk_group_bps.count(p.disk_group.at(hs.first))) return true;
      if (t != kDevice) {
        fanouts[hs.first].insert(fan);
        if (lm.second.limit_rate > 0) tier_capped[hs.first] = true;
      }
    }
  if (!p.link_bps.empty())  // a directed link shared by several of a sender's tiers
    for (auto& kv : sd_tiers)
      if (kv.second.size() > 1) {
        auto lk = p.link_bps.find(kv.first);
        if (lk != p.link_bps.end() && lk->second > 0) return true;
      }
  // A load-once budget (staging; tier rates with stage_once) over layers with
  // different fan-outs: the flow's fan-out scaling is exact only for one fan-out.
  for (auto& kv : fanouts) {
    if (kv.second.size() < 2) continue;
    auto st = p.stage_bps.find(kv.first);
    if ((st != p.stage_bps.end() && st->second > 0) || (p.stage_once && tier_capped[kv.first])) return true;
  }
  return false;
}

int64_t max_flow_at(const FlowProblem& p, double T) {
  Built b = build(p, T);
  return b.d->run(b.src, b.sink);
}

FlowPlan solve_flow(const FlowProblem& p) {
  if (needs_lp(p)) return solve_flow_lp(p);
  trace::Scoped tr("dissem.maxflow");
  FlowPlan plan;
  plan.solver = "flow";
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
  extract_jobs(per_demand, p.align, plan);
  return plan;
}

}  // namespace dissem
