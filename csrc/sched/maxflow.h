// Mode-3 planner: max-flow over (sender, tier) -> (layer, dest) with a search
// for the smallest completion time T (reference: distributor/flow.go:55-353).
//
// The reference builds a 6-tier graph on a dense V x V matrix and runs
// Edmonds-Karp, doubling then bisecting T over integer seconds, and supports
// one destination per layer (node.go:1078-1095). This planner:
//  * uses Dinic on a sparse residual graph (solved ~60x per plan);
//  * gives every (layer, dest) demand its own vertex, so a layer can go to many
//    destinations and each (sender, layer, dest) byte count is read directly
//    from one edge (quirk Q8);
//  * keeps one vertex per (sender, source tier) whose capacity is that tier's
//    rate (quirk Q7: the reference collapses every tier to SourceType 0);
//  * puts a per-sender staging vertex (host->HBM, PCIe) above its host, disk
//    and client tiers - bytes from those tiers cross the GPU's PCIe link before
//    any xGMI link, HBM-resident (Device) layers do not;
//  * optionally adds one vertex per directed link (sender -> dest) with its
//    capacity, shared by everything the sender sends to that dest: the xGMI
//    topology mode, where each GPU pair has one link. A sender whose layers for
//    one dest sit in several tiers gets one (tier, dest) vertex per tier instead,
//    each with the link's capacity split by that tier's share of the demanded
//    bytes (a link shared across tiers is a two-commodity constraint a single
//    flow cannot state exactly; the split keeps the plan feasible, never
//    optimistic - tests/test_maxflow.py checks both cases against an LP);
//  * searches T continuously (seconds as double), or over integer seconds for
//    reference parity;
//  * rounds byte counts to a chunk alignment so ranges map onto whole chunks.
//
// Constraints a single-commodity flow cannot state exactly - one directed link
// shared by layers from several of a sender's tiers, a staging (PCIe) budget
// paid once per loaded byte while layers fan out to different numbers of
// dests, one NVMe shared by every sender of a node (disk groups) - are solved
// as a linear program instead (sched/lp.h): min T over byte counts x[sender,
// class, dest] and loaded bytes y[sender, class] >= x, with every budget a
// rate * T row. Layers with the same holders (and tiers) and the same dests
// form one class, which keeps the LP small; its optimum equals the per-layer
// LP's. solver = "auto" uses the flow where it is exact and the LP otherwise.
#pragma once

#include <string>

#include <map>
#include <vector>

#include "core/types.h"

namespace dissem {

struct FlowDemand {
  LayerID layer;
  NodeID dest;
  int64_t size;
};

struct FlowJob {
  NodeID sender;
  LayerID layer;
  NodeID dest;
  int64_t size;
  int64_t offset;
};

struct FlowProblem {
  std::map<NodeID, int64_t> egress_bps;   // per sender NIC/link budget; 0 or absent = unlimited
  std::map<NodeID, int64_t> ingress_bps;  // per receiver; 0 or absent = unlimited
  std::map<NodeID, LayerIDs> holdings;    // what each potential sender holds (tier + rate)
  std::vector<FlowDemand> demands;
  std::map<std::pair<NodeID, NodeID>, int64_t> link_bps;  // optional per directed link caps
  std::map<NodeID, int64_t> stage_bps;   // per sender host->HBM staging (PCIe) for non-Device tiers
  int64_t align = 1;
  bool integer_seconds = false;
  bool allow_self = false;  // may a dest source a demand from its own lower tier
  // Planned (GPU) engines: a sender loads each byte of a non-HBM layer into
  // HBM once and forwards it to any number of dests, so its tier rate, its
  // staging budget and its disk group are charged per loaded byte, not per
  // transfer (the reference re-reads a layer for every transfer).
  bool stage_once = false;
  // Senders that read their disk tier from one shared device (one NVMe per
  // MI355X node): sender -> group, group -> read rate (B/s) shared by all.
  std::map<NodeID, int> disk_group;
  std::map<int, int64_t> disk_group_bps;
  // Planned engines: dests that load a layer from their own lower tier (mode-3
  // self-jobs, node.go:1205-1217) - layer -> bytes. The LP charges that load
  // to the dest's tier, staging and disk group, shared with whatever the dest
  // forwards of the same layer to others.
  std::map<NodeID, std::map<LayerID, int64_t>> self_loads;
  // Several hosts: node -> host, and each node's NIC rate (B/s, per direction)
  // that bounds what it sends to and receives from nodes of OTHER hosts (one
  // NIC per GPU; traffic inside a host rides its xGMI links). Solved by the LP.
  std::map<NodeID, int> host;
  std::map<NodeID, int64_t> nic_bps;
  std::string solver = "auto";  // "flow", "lp" or "auto"
};

struct FlowPlan {
  double T = 0;            // seconds
  int64_t required = 0;
  int64_t max_flow = 0;
  int solves = 0;
  bool feasible = false;
  std::string solver;      // "flow" or "lp"
  int lp_pivots = 0;
  std::string lp_status;   // the LP's outcome ("optimal", "infeasible", "iteration limit", ...)
  std::vector<FlowJob> jobs;
};

FlowPlan solve_flow(const FlowProblem& p);

// Max-flow only (exposed for tests): returns max flow for a fixed T.
int64_t max_flow_at(const FlowProblem& p, double T);
// Does `p` need the LP for an exact answer (see above)?
bool needs_lp(const FlowProblem& p);

}  // namespace dissem
