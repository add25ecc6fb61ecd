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
#pragma once

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
};

struct FlowPlan {
  double T = 0;            // seconds
  int64_t required = 0;
  int64_t max_flow = 0;
  int solves = 0;
  bool feasible = false;
  std::vector<FlowJob> jobs;
};

FlowPlan solve_flow(const FlowProblem& p);

// Max-flow only (exposed for tests): returns max flow for a fixed T.
int64_t max_flow_at(const FlowProblem& p, double T);

}  // namespace dissem
