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

// Dinic on a sparse residual graph whose capacities are affine in T: an edge
// carries fixed + floor(rate * T) bytes, or is unbounded. The graph is built
// once per plan; each T re-sets the capacities and re-runs the flow, and the
// source side of the final residual graph is a minimum cut, whose fixed and
// rate parts drive the parametric search for T (solve_flow below).
struct Dinic {
  struct E {
    int to;
    int64_t cap;
  };
  struct P {  // capacity parameters of a forward edge
    double rate = 0;
    int64_t fixed = 0;
    bool inf = false;
  };
  std::vector<E> e;
  std::vector<P> par;  // per forward edge (index id / 2)
  std::vector<std::vector<int>> g;
  std::vector<int> level, it;
  explicit Dinic(int n) : g(size_t(n)), level(size_t(n)), it(size_t(n)) {}
  int add(int u, int v, P prm) {
    e.push_back({v, 0});
    g[size_t(u)].push_back(int(e.size()) - 1);
    e.push_back({u, 0});
    g[size_t(v)].push_back(int(e.size()) - 1);
    par.push_back(prm);
    return int(e.size()) - 2;
  }
  static int64_t cap_at(const P& q, double T) {
    if (q.inf) return kInf;
    const double c = double(q.fixed) + std::floor(q.rate * T);
    return c >= 4e18 ? kInf : int64_t(c);
  }
  void set_T(double T) {
    for (size_t i = 0; i < par.size(); ++i) {
      e[2 * i].cap = cap_at(par[i], T);
      e[2 * i + 1].cap = 0;
    }
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
    return flow;  // `level` now marks the source side of a minimum cut
  }
  // The minimum cut left by run(): its fixed bytes, its rate (B/s of T) and
  // its edge count; false if an unbounded edge crosses it.
  bool cut(double* fixed, double* rate, int* edges) const {
    *fixed = *rate = 0;
    *edges = 0;
    for (size_t i = 0; i < par.size(); ++i) {
      const int u = e[2 * i + 1].to, v = e[2 * i].to;
      if (level[size_t(u)] < 0 || level[size_t(v)] >= 0) continue;
      if (par[i].inf) return false;
      *fixed += double(par[i].fixed);
      *rate += par[i].rate;
      ++*edges;
    }
    return true;
  }
  int64_t flow_on(int id) const { return e[size_t(id ^ 1)].cap; }
};

Dinic::P unlimited() { return Dinic::P{0, 0, true}; }
Dinic::P fixed_bytes(int64_t b) { return Dinic::P{0, b, false}; }
// rate <= 0: unlimited (the reference's LimitRate 0, quirk Q1)
Dinic::P per_second(double rate) { return rate > 0 ? Dinic::P{rate, 0, false} : unlimited(); }

int64_t required_bytes(const FlowProblem& p) {
  std::map<std::pair<LayerID, NodeID>, int64_t> dsize;
  for (auto& dm : p.demands) dsize[{dm.layer, dm.dest}] = std::max(dsize[{dm.layer, dm.dest}], dm.size);
  int64_t r = 0;
  for (auto& kv : dsize) r += kv.second;
  return r;
}

// Layers with the same holders (and tiers) and the same demands (dest, bytes):
// one class. Every layer of a class has the same constraints in the flow and
// in the LP, so both solve over classes (80 layers with one random holder
// each are 8 classes at 8 ranks) and split a class's bytes back onto its
// layers (split_class below) - the optimum is the per-layer problem's.
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

// One class's bytes for one dest, per sender (sender order = ascending id),
// cut into per-layer ranges. The class's layers are laid end to end as one
// stream of L x size bytes and each sender takes the next run of its share,
// with every cut rounded to the chunk grid inside its layer: most layers
// come whole from one sender and a share splits at most the two layers at
// its ends (L + senders pieces, not L x senders). A sender that serves
// several dests of a class the same share sends each of them the same region,
// so it loads those bytes once. The ranges partition every layer exactly.
void split_class(const LpClass& c, NodeID dest, int64_t size, std::vector<std::pair<NodeID, int64_t>> shares,
                 int64_t align, FlowPlan& plan) {
  const int64_t L = int64_t(c.layers.size());
  const int64_t total = L * size;
  if (total <= 0) return;
  std::sort(shares.begin(), shares.end());
  shares.erase(std::remove_if(shares.begin(), shares.end(), [](auto& x) { return x.second <= 0; }), shares.end());
  if (shares.empty()) return;
  int64_t sum = 0;
  for (auto& x : shares) sum += x.second;
  // integer bytes: the shares add up to the class demand (remainder to the biggest)
  size_t big = 0;
  for (size_t i = 1; i < shares.size(); ++i)
    if (shares[i].second > shares[big].second) big = i;
  shares[big].second += total - sum;
  const int64_t a = std::max<int64_t>(align, 1);
  auto snap = [&](int64_t q) {  // a cut at stream position q, on the grid of its layer
    if (q <= 0 || q >= total) return std::min(std::max<int64_t>(q, 0), total);
    const int64_t li = q / size, off = q - li * size;
    int64_t r = (off + a / 2) / a * a;
    if (r > size) r = size;
    if (size - r < a / 2 && size - r < r - off + a) r = size;  // the layer's short last chunk stays whole
    return li * size + r;
  };
  int64_t pos = 0, acc = 0;
  for (size_t k = 0; k < shares.size(); ++k) {
    acc += shares[k].second;
    const int64_t end = k + 1 == shares.size() ? total : std::max(pos, snap(acc));
    for (int64_t q = pos; q < end;) {
      const int64_t li = q / size, off = q - li * size;
      const int64_t n = std::min(end - q, size - off);
      plan.jobs.push_back(FlowJob{shares[k].first, c.layers[size_t(li)], dest, n, off});
      q += n;
    }
    pos = end;
  }
}

// The parametric flow graph: vertices per class demand instead of per layer.
struct FlowGraph {
  std::unique_ptr<Dinic> d;
  int src = 0, sink = 1;
  struct Job {
    NodeID s;
    size_t cls;
    NodeID dst;
    int edge;
  };
  std::vector<Job> jobs;
};

FlowGraph build(const FlowProblem& p, const std::vector<LpClass>& classes) {
  const bool topo = !p.link_bps.empty();
  const int kDevice = int(SourceType::Device);
  struct Cand {
    NodeID s;
    int t;
    size_t c;
    NodeID d;
    int64_t bytes;  // the class's demand at d
  };
  std::vector<Cand> cands;
  // per (sender, dest): demanded bytes by tier (to split a link shared by several tiers)
  std::map<std::pair<NodeID, NodeID>, std::map<int, int64_t>> sd_tiers;
  std::map<NodeID, double> cand_bytes, layer_bytes;  // staging fan-out per sender
  for (size_t ci = 0; ci < classes.size(); ++ci) {
    const LpClass& c = classes[ci];
    const int64_t L = int64_t(c.layers.size());
    int64_t mx = 0;
    for (auto& dz : c.dests) mx = std::max(mx, dz.second);
    for (auto& h : c.holders) {
      bool any = false;
      for (auto& dz : c.dests) {
        if (dz.first == h.first && !p.allow_self) continue;
        const int64_t b = dz.second * L;
        cands.push_back({h.first, h.second, ci, dz.first, b});
        sd_tiers[{h.first, dz.first}][h.second] += b;
        if (h.second != kDevice) cand_bytes[h.first] += double(b);
        any = true;
      }
      if (any && h.second != kDevice) layer_bytes[h.first] += double(mx * L);
    }
  }
  int n = 2;
  std::map<NodeID, int> vs, vstage, vdest;
  std::map<std::pair<NodeID, int>, int> vst;
  std::map<std::tuple<NodeID, int, NodeID>, int> vlink;  // (s, tier or -1 = shared, d)
  std::map<std::pair<size_t, NodeID>, int> vd;
  std::map<std::pair<size_t, NodeID>, int64_t> vd_bytes;
  for (auto& c : cands) {
    if (!vd.count({c.c, c.d})) {
      vd[{c.c, c.d}] = n++;
      vd_bytes[{c.c, c.d}] = c.bytes;
    }
    if (!vdest.count(c.d)) vdest[c.d] = n++;
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
  FlowGraph b;
  b.d = std::make_unique<Dinic>(n);
  Dinic& d = *b.d;
  auto rate_of = [](const std::map<NodeID, int64_t>& m, NodeID k) {
    auto it = m.find(k);
    return it == m.end() ? int64_t(0) : it->second;
  };
  for (auto& kv : vs) d.add(b.src, kv.second, per_second(double(rate_of(p.egress_bps, kv.first))));
  // Staging is paid once per byte a sender loads into HBM, however many dests it
  // then forwards it to over xGMI; a flow charges every transfer, so the
  // budget is scaled by the sender's fan-out (its candidate bytes over the
  // distinct layer bytes it could load) - exact when its layers share one
  // fan-out (needs_lp sends the other cases to the LP).
  auto fan = [&](NodeID s) {
    return layer_bytes[s] > 0 ? std::max(1.0, cand_bytes[s] / layer_bytes[s]) : 1.0;
  };
  for (auto& kv : vstage) {
    const int64_t r = rate_of(p.stage_bps, kv.first);
    d.add(vs[kv.first], kv.second, r > 0 ? per_second(double(r) * fan(kv.first)) : unlimited());
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
    double r = double(tier_rate[kv.first]);
    if (p.stage_once && !dev && r > 0) r *= fan(s);  // read once, forwarded to every dest
    d.add(parent, kv.second, per_second(r));
  }
  for (auto& kv : vlink) {
    const NodeID s = std::get<0>(kv.first), dst = std::get<2>(kv.first);
    const int t = std::get<1>(kv.first);
    auto lk = p.link_bps.find({s, dst});
    double rate = lk == p.link_bps.end() ? 0.0 : double(lk->second);
    const auto& tiers = sd_tiers[{s, dst}];
    if (t >= 0 && rate > 0) {
      // several tiers share this link: each gets its share of the demanded bytes
      int64_t tot = 0;
      for (auto& x : tiers) tot += x.second;
      if (tot > 0) rate *= double(tiers.at(t)) / double(tot);
    }
    // a shared vertex is fed by every tier of the sender that serves this dest
    const int from = t >= 0 ? vst[{s, t}] : vst[{s, tiers.begin()->first}];
    d.add(from, kv.second, per_second(rate));
  }
  for (auto& c : cands) {
    const int from = (topo && c.s != c.d) ? vlink[link_key(c)] : vst[{c.s, c.t}];
    b.jobs.push_back({c.s, c.c, c.d, d.add(from, vd[{c.c, c.d}], unlimited())});
  }
  for (auto& kv : vd) d.add(kv.second, vdest[kv.first.second], fixed_bytes(vd_bytes[kv.first]));
  for (auto& kv : vdest) d.add(kv.second, b.sink, per_second(double(rate_of(p.ingress_bps, kv.first))));
  return b;
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
  // Class bytes back to layers: per (class, dest) the senders' shares, cut into ranges.
  std::map<std::pair<size_t, NodeID>, std::vector<std::pair<NodeID, int64_t>>> shares;
  for (size_t i = 0; i < xs.size(); ++i) {
    const double bytes = r.x[size_t(xs[i].col)] * B0;
    shares[{xs[i].c, xs[i].d}].push_back({xs[i].s, int64_t(std::llround(std::max(0.0, bytes)))});
  }
  for (size_t ci = 0; ci < classes.size(); ++ci)
    for (auto& dz : classes[ci].dests) split_class(classes[ci], dz.first, dz.second, shares[{ci, dz.first}], p.align, plan);
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
  const auto classes = lp_classes(p);
  FlowGraph b = build(p, classes);
  b.d->set_T(T);
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
  const auto classes = lp_classes(p);
  FlowGraph b = build(p, classes);
  Dinic& d = *b.d;
  const double D = double(plan.required);
  auto flow = [&](double T) {
    ++plan.solves;
    d.set_T(T);
    return d.run(b.src, b.sink);
  };
  // Parametric search (Newton / Dinkelbach on the min cut): the max flow at T
  // is the minimum over cuts of fixed + rate * T, concave and piecewise
  // linear. From a T below the optimum, the minimum cut at T reaches the
  // demand at T' = (D - fixed) / rate, which is still <= the optimum; every
  // step moves to a new cut of the optimum's envelope, so a few max-flows
  // (not the reference's ~60-step doubling + bisection, flow.go:155-191) give
  // the smallest T exactly. The floor of each edge's rate * T loses < 1 byte,
  // so a step adds one byte per cut edge.
  double T = 1e-12;
  int64_t f = flow(T);
  for (int it = 0; f < plan.required && it < 256; ++it) {
    double fixed = 0, rate = 0;
    int edges = 0;
    if (!d.cut(&fixed, &rate, &edges) || rate <= 0) break;  // no T-dependent edge: infeasible
    const double Tn = (D - fixed + double(edges)) / rate;
    if (!(Tn > T)) {  // rounding: nudge up
      T = T * (1 + 1e-12) + 1e-15;
    } else {
      T = Tn;
    }
    f = flow(T);
  }
  if (f < plan.required) return plan;  // infeasible (some demand has no holder)
  if (p.integer_seconds) {
    // the reference's integer-second search (flow.go:171-187) = the smallest whole second >= T
    double Ti = std::max(1.0, std::ceil(T * (1 - 1e-12) - 1e-9));
    while (flow(Ti) < plan.required) Ti += 1;
    T = Ti;
    f = flow(T);
  }
  plan.max_flow = f;
  plan.T = T;
  plan.feasible = true;
  std::map<std::pair<size_t, NodeID>, std::vector<std::pair<NodeID, int64_t>>> shares;
  for (auto& j : b.jobs) {
    const int64_t x = d.flow_on(j.edge);
    if (x > 0) shares[{j.cls, j.dst}].push_back({j.s, x});
  }
  for (size_t ci = 0; ci < classes.size(); ++ci)
    for (auto& dz : classes[ci].dests) split_class(classes[ci], dz.first, dz.second, shares[{ci, dz.first}], p.align, plan);
  return plan;
}

}  // namespace dissem
