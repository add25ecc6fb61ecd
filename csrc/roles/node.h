// Roles: leader (coordinator) and receiver state machines for distribution
// modes 0-3, plus the external client (reference: distributor/node.go,
// client.go).
//
// The reference builds a class hierarchy (LeaderNode -> RetransmitLeaderNode ->
// Pull/Flow leaders, ReceiverNode -> Retransmit/Flow receivers) and spawns a
// goroutine per message, guarding shared maps with RWMutexes (several of which
// race). Here one Node owns all role state and processes its inbox
// on a single event-loop thread; a leader is a Node with `is_leader` set, and
// every node (the leader included) can act as a sender or receiver. Mode policy
// lives in small strategy functions (mode0/1/2/3 in node.cc).
#pragma once

#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <thread>

#include "core/vclock.h"
#include "engine/engine.h"
#include "store/store.h"
#include "transport/transport.h"

namespace dissem {

struct NodeConfig {
  NodeID id = 0;
  NodeID leader = 0;
  int mode = 0;                     // 0 naive, 1 retransmit, 2 pull, 3 flow
  uint64_t epoch = 0;               // session id carried in messages (0 = none)
  uint64_t seed = 0;                // mode-1 owner RNG (quirk Q5: seeded uniform choice)
  std::string owner_policy = "random";  // mode 1: "random" (reference), "balanced" (egress), "links" (per-link)
  int pull_window = 1;              // mode 2: concurrent jobs per sender (reference: 1)
  int64_t pull_job_bytes = 0;       // mode 2: job = this many bytes of a layer (0 = whole layer, reference)
  bool range_acks = false;          // receiver: also ack each landed range (needed by mode-2 range jobs)
  std::map<NodeID, int64_t> network_bw;  // mode 3: NetworkBW per node (B/s, 0 = unlimited)
  std::map<std::pair<NodeID, NodeID>, int64_t> link_bw;  // mode 1 links / mode 3 topology: per directed link
  std::map<NodeID, int64_t> stage_bw;  // mode 3: per node host->HBM staging (PCIe) budget for non-HBM tiers
  std::map<NodeID, int64_t> hbm_bw;    // mode 3: per node HBM ingress (write) budget; min'd with NetworkBW
  bool integer_seconds = false;     // mode 3: reference T search over integer seconds
  int64_t align = 1;                // mode 3: byte alignment of ranges
  std::string storage_path;         // receiver persist dir ("" = none)
  bool relay = true;                // planned mode 0: scatter + peer relay instead of leader fan-out
  bool collective = false;          // planned mode 0: ncclBroadcast when every other rank needs the layer
  // Failure handling (the reference waits forever for a dead
  // sender's ack). Leader, host engines: a job not acked within
  // job_timeout_s + bytes/job_min_rate is re-dispatched from another owner and
  // its sender is suspected (no new jobs). 0 = off (reference behavior).
  double job_timeout_s = 0;
  double job_min_rate = 0;          // B/s allowance added to the deadline (0 = flat timeout)
  int max_redispatch = 8;           // per (dest, layer, range)
  // Closed-loop link rates: this node's measured outbound rate to each peer
  // (B/s; e.g. an EWMA of earlier sessions' per-link busy throughput or the
  // pre-flight probe), sent with its announce. With adapt_links the leader
  // plans on every node's reported rates instead of link_bw's estimates:
  // mode-1 "links" owners and relays, mode-3 capacities and T, mode-2 sender
  // choice (reference: node.go:774-793 measures job times, :1044-1053 uses them).
  std::map<NodeID, int64_t> link_report;     // closed loop: this node's measured rate to each peer (B/s)
  std::map<NodeID, int64_t> link_report_in;  // ... and each peer's link into this node, timed here
  bool adapt_links = true;
  // Nodes whose disk tiers read one shared device (all ranks of one MI355X
  // node share its NVMe): node -> group, group -> read rate (B/s). Mode 3 plans
  // the group as one budget (sched/maxflow.h).
  std::map<NodeID, int> disk_group;
  std::map<int, int64_t> disk_group_bw;
  // Planned mode 0 (BASELINE config #2 from host memory): the leader's host
  // layers sit in node-shared pinned memory that every rank has mapped, so
  // every rank holding a layer's bytes stages a 1/k slice of it over its own
  // PCIe and sends that slice to every dest - k host links feed the xGMI mesh
  // instead of the leader's one (reference mode 0: the leader pushes
  // everything, node.go:326-352; that stays the default).
  bool host_share = false;
  // Multi-node runs: node -> host (GPUs of one host share an xGMI mesh; hosts
  // are joined by one NIC per GPU). Empty / one value: a single host. With
  // several, mode 1's "links" policy imports a layer once per host and relays
  // it inside the host (Node::schedule_imports).
  std::map<NodeID, int> host;
  std::map<NodeID, int64_t> nic_bw;  // several hosts: each node's NIC (B/s per direction), mode 3's budget
};

struct NodeStats {
  double time_to_deliver_s = 0;  // leader: start -> assignment satisfied
  int64_t bytes_planned = 0;     // leader: bytes that had to move at start
  int64_t jobs_dispatched = 0;
  int64_t layers_received = 0;
  int64_t bytes_received = 0;
  double flow_T = 0;             // mode 3 planned completion time (s)
  double plan_ms = 0;            // leader: scheduling time (plan + dispatch of the transfer batches)
  double plan_sched_ms = 0;      // leader: of which the scheduler (or the plan cache lookup)
  double plan_dispatch_ms = 0;   // leader: of which encoding + sending the transfer batches
  bool plan_cached = false;      // leader: the plan was an identical earlier session's (roles/plan_cache.h)
  std::string plan_solver;       // leader: which scheduler / solver planned ("mode1:links", "flow", "lp", ...)
  int64_t plan_gap_bytes = 0;    // leader, mode 3: bytes the plan left uncovered (an invariant violation; 0)
  int64_t nacks = 0;             // leader: chunk re-sends requested by receivers (CRC mismatch)
  int64_t redispatched = 0;      // leader: jobs re-sent from another owner after their deadline
  int64_t suspects = 0;          // leader: senders that missed a deadline
  int64_t recoveries = 0;        // leader: communicator shrinks after a rank died (planned engines)
  int64_t dropped = 0;           // leader: (dest, layer) pairs given up (dead dest or no live owner)
};

class Node {
 public:
  Node(NodeConfig cfg, std::shared_ptr<Transport> t, std::shared_ptr<DataEngine> e, const LayersSrc& layers,
       const Assignment& assignment, bool is_leader);
  ~Node();

  void start();
  void stop();

  // Receiver API (node.go:1291-1297).
  void announce();
  bool wait_ready(double timeout_s);
  // Leader API (node.go:214-226).
  bool wait_start(double timeout_s);
  Assignment assignment() const { return assignment_; }
  Status status();
  NodeStats stats();

  // Routing (node.go:17-122): 1-hop table; updateLeader kept for failover.
  void add_node(NodeID goal) { add_routing(goal, goal, 1); }
  void add_routing(NodeID goal, NodeID next_hop, unsigned hops);
  NodeID next_hop(NodeID goal);
  void update_leader(NodeID leader);
  // Leader: the per directed link rates the last plan used (B/s).
  std::map<std::pair<NodeID, NodeID>, int64_t> plan_link_bw();

  // Accessors for engines.
  NodeID id() const { return cfg_.id; }
  NodeID leader() const { return cfg_.leader; }
  uint64_t epoch() const { return cfg_.epoch; }
  Transport* transport() { return t_.get(); }
  LayerStore& store() { return store_; }
  DataEngine* engine() { return e_.get(); }
  void inject(MessagePtr m) { t_->inject(std::move(m)); }
  // Safe send from any thread (logs on failure).
  bool send_msg(NodeID dest, Message m);
  // Ask this node's external client to stream `layer` here (any thread): the
  // planned engine's way to obtain a client-held layer before it can stage it.
  void request_client_layer(LayerID layer);
  bool is_leader() const { return is_leader_; }

 private:
  void loop();
  void handle(const MessagePtr& m);
  // receiver-side
  void on_layer(const MessagePtr& m);
  void on_landed(LayerID layer, int64_t off, int64_t size, int64_t total, NodeID from, double dur_ms);
  void on_retransmit(const MessagePtr& m);
  void on_flow_retransmit(const MessagePtr& m);
  void on_startup(const MessagePtr& m);
  void send_ack(LayerID layer);
  // sender-side
  void send_layer(NodeID dest, LayerID layer, int64_t offset, int64_t size, int64_t rate);
  void fetch_from_client(LayerID layer, NodeID dest);
  // leader-side
  void on_announce(const MessagePtr& m);
  void merge_link_rates(NodeID src, const std::map<NodeID, int64_t>& out, const std::map<NodeID, int64_t>& in);
  void on_ack(const MessagePtr& m);
  bool assignment_satisfied();
  void send_startup();
  void start_distribution();
  // failure handling (leader)
  void on_nack(const MessagePtr& m);
  // elastic recovery of the planned data plane (leader)
  void on_suspect(const MessagePtr& m);
  void on_shrink_done(const MessagePtr& m);
  void replan_after_shrink();
  void finish_if_satisfied();
  void on_tick();
  void track(NodeID sender, NodeID dest, LayerID layer, int64_t off, int64_t size);
  NodeID alternative_owner(LayerID layer, NodeID dest, NodeID avoid);
  void ticker();
  int64_t layer_size(LayerID l);
  std::string plan_key();
  void retransmit(LayerID layer, NodeID owner, NodeID dest);
  void add_job(NodeID src, NodeID dst, LayerID layer, int64_t offset, int64_t size, int phase = 0, int64_t rate = 0);
  void flush_batch();
  void schedule_mode0();
  void schedule_mode1();
  struct PlanPart {
    NodeID src;
    int64_t off, size;
    int phase;  // 0: from an owner, 1: relayed by a rank that receives the layer in phase 0
  };
  using RelayPlan = std::map<std::pair<NodeID, LayerID>, std::vector<PlanPart>>;  // (dest, layer) -> parts
  void relay_rebalance(RelayPlan& plan, const std::function<double(NodeID, NodeID)>& cap);
  // multi-host (cfg_.host): (host, layer) -> dests of that host needing the layer + their missing ranges
  using ImportMap =
      std::map<std::pair<int, LayerID>, std::vector<std::pair<NodeID, std::vector<std::pair<int64_t, int64_t>>>>>;
  void schedule_imports(const ImportMap& imports, RelayPlan& plan, const std::function<double(NodeID, NodeID)>& cap);
  void relay_across_hosts(LayerID layer, int64_t total, const std::vector<NodeID>& remote, std::map<int, int64_t>& rot);
  int host_of(NodeID n) const;
  bool multi_host() const;
  void schedule_mode2();
  void schedule_mode3();
  // mode 2 (node.go:628-1073); a job is (layer, dest, byte range)
  using JobKey = std::pair<NodeID, int64_t>;  // (dest, offset) within jobs_[layer]
  bool assign_new_job(NodeID node, bool steal = true);
  NodeID min_loaded_sender(LayerID layer, NodeID dest);
  bool rarest_own_job(NodeID node, LayerID* layer, JobKey* key);
  bool rarest_stealable_job(NodeID node, LayerID* layer, JobKey* key, NodeID* victim);
  void dispatch_range(LayerID layer, NodeID sender, NodeID dest, int64_t off, int64_t size);
  void retire_job(LayerID layer, const JobKey& key);
  void on_range_ack(const MessagePtr& m);

  NodeConfig cfg_;
  std::shared_ptr<Transport> t_;
  std::shared_ptr<DataEngine> e_;
  LayerStore store_;
  Assignment assignment_;
  bool is_leader_;
  std::thread loop_th_;
  std::atomic<bool> running_{false};

  std::mutex rt_mu_;
  std::map<NodeID, std::pair<NodeID, unsigned>> routing_;

  // leader state (event-loop thread only, except where noted)
  Status status_;
  std::map<LayerID, NodeIDs> owners_;
  std::mt19937_64 rng_;
  std::map<NodeID, int64_t> owner_bytes_;  // balanced owner policy
  std::map<std::pair<NodeID, NodeID>, int64_t> link_bytes_;  // "links" owner policy: bytes per (src, dst)
  enum class JobState { Pending, Sending };
  struct Job {
    NodeID sender = 0;
    JobState state = JobState::Pending;
    int64_t t_us = 0;
    int64_t size = 0;  // range [key.second, key.second + size)
    RangeSet got;      // bytes the dest reported landed (range acks)
  };
  std::map<LayerID, std::map<JobKey, Job>> jobs_;
  std::map<NodeID, int64_t> load_;        // senderLoadCounter
  std::map<NodeID, int> inflight_;        // jobs currently sending per sender (network jobs)
  // planned engines: a sender's loads of its own layers in flight, a window of
  // their own beside the network one (mode2.cc, kSelfWindow)
  std::map<NodeID, int> self_inflight_;
  bool self_job(NodeID sender, NodeID dest) const { return sender == dest && e_->planned(); }
  bool job_room(NodeID sender, NodeID dest);
  int& job_slots(NodeID sender, NodeID dest) { return (self_job(sender, dest) ? self_inflight_ : inflight_)[sender]; }
  std::map<NodeID, std::pair<double, uint64_t>> perf_;  // sender -> (EWMA job us, count) (quirk Q9)
  // planned data plane (leader): jobs awaiting dispatch, sequence numbers, CRC manifests
  struct PendingJob {
    XferJob job;
    int phase;
  };
  std::vector<PendingJob> pending_jobs_;
  uint64_t next_seq_ = 1, next_batch_ = 1;
  std::map<std::pair<NodeID, NodeID>, int64_t> measured_links_;  // leader: merged link rates (B/s, merged_link_rates)
  // leader: per directed link, the sender's report (timed at the sending end)
  // and the receiver's (timed at the receiving end)
  std::map<std::pair<NodeID, NodeID>, int64_t> reported_out_, reported_in_;
  void merged_link_rates();
  std::map<LayerID, CrcManifest> manifests_;  // whole copies' manifests
  std::map<LayerID, std::set<NodeID>> manifest_holders_;  // who announced a whole copy's manifest
  // chunk CRCs vouched for by partial copies: layer -> (grid, chunk -> crc)
  std::map<LayerID, std::pair<int64_t, std::map<int64_t, uint32_t>>> partial_crc_;
  void merge_partial_manifest(LayerID layer, const CrcManifest& m,
                              const std::vector<std::pair<int64_t, int64_t>>& ranges);
  // failure handling (leader, event-loop thread)
  struct Outstanding {
    NodeID sender;
    int64_t off, size, t_us;
  };
  std::map<std::pair<NodeID, LayerID>, std::vector<Outstanding>> outstanding_;  // (dest, layer)
  std::map<std::tuple<NodeID, LayerID, int64_t>, int> redispatches_;
  std::set<NodeID> suspects_;
  Status initial_status_;  // inventories at start (re-send sources for NACKs)
  uint64_t shrink_gen_ = 0;         // recovery generation
  std::set<NodeID> dead_nodes_;     // confirmed dead (liveness probe failed)
  std::set<NodeID> shrink_wait_;    // survivors whose ShrinkDone is outstanding
  std::thread tick_th_;
  std::mutex tick_mu_;
  CondVar tick_cv_;
  bool tick_stop_ = false;

  // cross-thread signalling
  std::mutex sig_mu_;
  CondVar sig_cv_;
  bool started_ = false, satisfied_ = false, ready_ = false;
  int64_t t_start_us_ = 0, t_ready_us_ = 0;  // vclock::now_us (model time in simulations)
  uint64_t session_range_ = 0;  // roctx range: timer start -> assignment satisfied
  NodeStats stats_;
  std::set<LayerID> acked_;
  std::map<NodeID, PartialLayers> partial_;  // leader: announced partial copies (chunk-granular resume)
  std::mutex stream_mu_;  // reader threads of the transport
  std::map<LayerID, int64_t> stream_prefix_;  // cut-through: host bytes of a client stream handed to the engine
};

// External client: a separate process holding rate-limited layers in memory
// that streams a layer to its node on ClientReq (reference: client.go).
class ClientNode {
 public:
  ClientNode(NodeID node_id, std::shared_ptr<Transport> t, const LayersSrc& layers);
  ~ClientNode();
  void start();
  void stop();

 private:
  NodeID node_id_;
  std::shared_ptr<Transport> t_;
  LayersSrc layers_;
  std::thread th_;
  WorkerSet workers_;
};

}  // namespace dissem
