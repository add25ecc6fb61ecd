// Mode 3: flow-retransmit leader (reference: node.go:1200-1288 + flow.go) -
// self-jobs, then the max-flow / LP plan (sched/maxflow.h) dispatched as byte
// ranges paced at size / T.
#include "roles/node.h"

#include <algorithm>
#include <climits>
#include <set>
#include <tuple>

#include "core/log.h"
#include "core/trace.h"
#include "roles/node_internal.h"
#include "sched/maxflow.h"

namespace dissem {

// ------------------------------------------------------------------- mode 3

void Node::schedule_mode3() {
  // node.go:1200-1288 + flow.go
  FlowProblem p;
  const Location tgt = e_->target();
  std::vector<FlowDemand> demands;
  struct SelfJob {
    NodeID dest;
    LayerID layer;
    int64_t size, rate;
  };
  std::vector<SelfJob> self_jobs;
  for (auto& kv : assignment_) {
    for (auto& l : kv.second) {
      auto& st = status_[kv.first];
      if (at(st, l.first, tgt)) continue;
      auto it = st.find(l.first);
      if (it != st.end()) {
        self_jobs.push_back({kv.first, l.first, layer_size(l.first), it->second.limit_rate});
      } else {
        demands.push_back({l.first, kv.first, layer_size(l.first)});
      }
    }
  }
  for (auto& sj : self_jobs) {
    Message f;
    f.type = MsgType::FlowRetransmit;
    f.layer = sj.layer;
    f.dest = sj.dest;
    f.data_size = sj.size;
    f.offset = 0;
    f.rate = sj.rate;
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.jobs_dispatched++;
    }
    if (e_->planned()) {
      add_job(sj.dest, sj.dest, sj.layer, 0, sj.size);
    } else {
      track(sj.dest, sj.dest, sj.layer, 0, sj.size);
      send_msg(sj.dest, f);
    }
  }
  if (demands.empty()) {
    log::info(int64_t(cfg_.id)).msg("No jobs to assign other than self-assignment");
    return;
  }
  p.demands = demands;
  p.holdings = status_;
  for (auto& kv : cfg_.network_bw) {
    p.egress_bps[kv.first] = kv.second;
    p.ingress_bps[kv.first] = kv.second;
  }
  for (auto& kv : cfg_.hbm_bw) {
    if (kv.second <= 0) continue;
    auto it = p.ingress_bps.find(kv.first);
    if (it == p.ingress_bps.end() || it->second <= 0 || it->second > kv.second) p.ingress_bps[kv.first] = kv.second;
  }
  p.link_bps = cfg_.link_bw;
  p.stage_bps = cfg_.stage_bw;
  p.align = cfg_.align;
  p.integer_seconds = cfg_.integer_seconds;
  p.disk_group = cfg_.disk_group;
  p.disk_group_bps = cfg_.disk_group_bw;
  if (multi_host()) {
    p.host = cfg_.host;
    p.nic_bps = cfg_.nic_bw;
  }
  if (e_->planned()) {
    // GPU data plane: a layer is loaded into HBM once and forwarded from there;
    // a self-job's load feeds the dest's own sends of that layer too.
    p.stage_once = true;
    for (auto& sj : self_jobs) {
      auto st = status_[sj.dest].find(sj.layer);
      if (st != status_[sj.dest].end() && st->second.source_type != SourceType::Device)
        p.self_loads[sj.dest][sj.layer] = sj.size;
    }
  }
  log::info(int64_t(cfg_.id)).msg("assigning a job...");
  int64_t t0 = log::now_us();
  FlowPlan plan = solve_flow(p);
  std::string solver = plan.solver;
  if (!plan.feasible && plan.solver == "lp") {
    // The LP (sched/lp.cc) solves every instance of the wide-range test set
    // (tests/test_maxflow.py); reaching this branch is a planner defect, which
    // is logged as an error and counted (stats plan_solver "lp->flow"). The
    // session still runs on the flow plan: it relaxes the budgets it cannot
    // state, so its T may be optimistic, but every demand gets a sender.
    log::error(int64_t(cfg_.id)).s("lp_status", plan.lp_status).i("lp_pivots", plan.lp_pivots)
        .msg("mode 3: the LP failed, planning with the max-flow instead");
    p.solver = "flow";
    plan = solve_flow(p);
    solver = "lp->flow";
  }
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.plan_solver = solver;
  }
  log::info(int64_t(cfg_.id)).f("computation time[ms]", double(log::now_us() - t0) / 1e3).i("solves", plan.solves)
      .s("solver", plan.solver).i("lp_pivots", plan.lp_pivots).msg("Job assignment completed");
  log::info(int64_t(cfg_.id)).f("required minimum time(s)", plan.T).b("feasible", plan.feasible)
      .msg("job assignment calculated");
  {
    std::lock_guard<std::mutex> lk(sig_mu_);
    stats_.flow_T = plan.T;
  }
  // Invariant: every demand's byte ranges cover its layer exactly (the
  // planner's split_class partitions each class by construction). A gap
  // would leave its dest waiting forever, so it is checked here: counted
  // (stats plan_gap_bytes, tests assert 0), logged as an error and, so that
  // no session hangs on a planner defect, filled from the demand's largest
  // sender at the plan's pace.
  if (plan.feasible) {
    std::map<std::pair<LayerID, NodeID>, std::vector<std::pair<int64_t, int64_t>>> cover;
    std::map<std::pair<LayerID, NodeID>, std::pair<NodeID, int64_t>> biggest;
    for (auto& j : plan.jobs) {
      cover[{j.layer, j.dest}].push_back({j.offset, j.offset + j.size});
      auto& b = biggest[{j.layer, j.dest}];
      if (j.size > b.second) b = {j.sender, j.size};
    }
    int64_t filled = 0;
    for (auto& d : p.demands) {
      auto& v = cover[{d.layer, d.dest}];
      std::sort(v.begin(), v.end());
      int64_t pos = 0;
      std::vector<std::pair<int64_t, int64_t>> gaps;
      for (auto& r : v) {
        if (r.first > pos) gaps.push_back({pos, r.first});
        pos = std::max(pos, r.second);
      }
      if (pos < d.size) gaps.push_back({pos, d.size});
      auto bg = biggest.find({d.layer, d.dest});
      NodeID src = bg != biggest.end() ? bg->second.first : kClientID;
      if (src == kClientID)
        for (auto& hs : p.holdings)
          if (hs.first != d.dest && hs.second.count(d.layer)) {
            src = hs.first;
            break;
          }
      if (src == kClientID) continue;
      for (auto& g : gaps) {
        plan.jobs.push_back(FlowJob{src, d.layer, d.dest, g.second - g.first, g.first});
        filled += g.second - g.first;
      }
    }
    if (filled) {
      log::error(int64_t(cfg_.id)).i("gap_bytes", filled).msg("mode 3: the plan left bytes uncovered (planner defect); filled from a sender");
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.plan_gap_bytes += filled;
    }
  }
  for (auto& j : plan.jobs) {
    Message f;
    f.type = MsgType::FlowRetransmit;
    f.layer = j.layer;
    f.dest = j.dest;
    f.data_size = j.size;
    f.offset = j.offset;
    f.rate = plan.T > 0 ? int64_t(double(j.size) / plan.T) : 0;  // node.go:1281 (pace to finish together)
    {
      std::lock_guard<std::mutex> lk(sig_mu_);
      stats_.jobs_dispatched++;
    }
    if (e_->planned()) {
      add_job(j.sender, j.dest, j.layer, j.offset, j.size, 0, f.rate);
    } else {
      track(j.sender, j.dest, j.layer, j.offset, j.size);
      send_msg(j.sender, f);
    }
  }
}

}  // namespace dissem
