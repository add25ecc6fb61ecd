// Planned data engine: executes the leader's sequence-numbered transfer jobs
// (XferBatch) as grouped point-to-point rounds on a device backend.
//
// Execution model (replaces the reference's "goroutine + fresh TCP connection
// per layer", transport.go:267-275):
//  * The leader turns every scheduling decision (mode 0/1/2/3) into XferJobs
//    with global sequence numbers and sends each rank its share.
//  * Each job is cut into pieces on a fixed chunk grid. A rank orders its pieces
//    by the key (batch, chunk index within the layer, sequence number) - a key its
//    partner computes identically. Pieces go to comm lanes (lane_of: by ring
//    distance of the pair, the same lane on both ends; one RCCL communicator +
//    HIP stream per lane) and each lane issues its pieces in key order as
//    groups of at most one send and one recv per peer. With one lane a group is
//    an all-to-all round over every xGMI link; with world-1 lanes every link
//    pair progresses on its own, so a slow or late peer stalls only its lane.
//    Because every lane posts in one global key order, the schedule cannot
//    deadlock (planned_engine.cc).
//  * Pacing (reference writeWithLimit, transport.go:407-424): sends of a job
//    with a rate (mode 3: size/T, node.go:1281) and sends to a rate-capped
//    peer (--inject slow-link) are issued no faster than their token bucket
//    allows; staging from a tier with a LimitRate (Sources) is paced per tier
//    (node.go:1615-1624).
//  * Host-tier sources are staged chunk by chunk on the copy queue; a send
//    waits on its chunk's staging event, so PCIe staging and xGMI transfer
//    pipeline per chunk (the reference's pipe/tee, at chunk grain).
//  * Every landed chunk is CRC32C-checked on the verify queue against the
//    holder's announced manifest before the node acks it.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "core/vclock.h"
#include "engine/backend.h"
#include "engine/engine.h"
#include "engine/node_pacer.h"
#include "store/store.h"

namespace dissem {

struct PlannedConfig {
  int rank = 0;
  int world = 1;
  std::vector<NodeID> rank_nodes;  // rank -> node id
  int64_t chunk_bytes = 64ll << 20;
  bool verify = true;
  bool poison = true;              // zero non-seeded slots between sessions
  // P2P groups in flight per rank, split evenly over the lanes (at least 4
  // per lane): enough queued link time to hide the issue thread, few enough
  // that RCCL's proxy never runs out of op slots behind a dead peer (which
  // would block ncclGroupEnd on the host).
  int max_inflight_groups = 64;
  // Independent comm lanes (communicator + stream each; backend.h lane_of).
  // 0 = auto: one lane per directed link, so every xGMI link of a GPU sends or
  // receives on its own. One-distance lanes are also what keeps irregular
  // groups (mode 2, relays) safe on RCCL: with few channels RCCL runs a
  // group's ops in rounds of one distance each, so a multi-distance group can
  // wait on itself across ranks (SimTiming::p2p_rounds reproduces it).
  int lanes = 0;
  // Multi-node runs: the ranks sit in this many hosts of world / hosts GPUs
  // each, in rank order (backend.h host_lanes); 1 = one host.
  int hosts = 1;
  int host_lane_classes = 0;       // lanes per direction to each other host (backend.h host_lanes; 0 = auto)
  std::map<NodeID, int64_t> link_rate;  // cap this rank's sends to a node (B/s; slow-link injection)
  int group_peers = 1;             // ops per peer and direction per group
  int disk_readers = 4;            // NVMe reader threads (O_DIRECT pread into pinned bounce buffers)
  bool disk_o_direct = true;       // false: buffered preads (tests of the fallback reporting)
  int disk_ring = 8;               // pinned bounce buffers of chunk_bytes each
  // One NVMe shared by every rank of the node: > 0 paces this rank's disk
  // reads through a node-wide budget of this many B/s (engine/node_pacer.h),
  // shared by every process that uses the same node_disk_key.
  int64_t node_disk_rate = 0;
  std::string node_disk_key;
  // fp8 wire/storage format (core/fp8.h): layers are staged from bf16 sources
  // and packed on the copy queue; HBM slots, transfers and CRCs use the packed
  // chunk grid. chunk_bytes stays the SOURCE (bf16) chunk.
  int pack = 0;                    // 0 none, 1 fp8 e4m3fn block-scaled
  int pack_block = 128;            // elements per f32 scale
  // pack = fp8 only: every chunk that becomes resident (received or staged) is
  // also dequantized to bf16 into a second HBM slot of the layer by the fused
  // verify+unpack kernel - the CRC check and the dequantization in one pass
  // over the packed bytes (--store bf16). Every rank then holds the same bf16
  // image (the source rank too: it unpacks its own packed chunks).
  bool unpack_store = false;
  // Fault handling: a chunk that fails its CRC is NACKed to the
  // leader, which re-sends it; after max_retries failures of one chunk the
  // engine fails. inject_corrupt overwrites received chunks with this
  // probability (fault injection, --inject drop-chunk=P).
  int max_retries = 4;
  double inject_corrupt = 0;
  uint64_t inject_seed = 1;
  double group_timeout_s = 300;    // a P2P group pending longer than this fails the engine (dead peer)
  // Elastic recovery (node-bound engines): a group pending longer than
  // suspect_s, or failing, is reported to the leader (Suspect); the leader
  // probes the peers and, if one is dead, has every survivor shrink the
  // communicator (Shrink) and re-plans the rest. 0 = report only on failure.
  double suspect_s = 10;
  int inject_die_after_groups = 0;  // fault injection: stop dead after this many groups (tests)
  // CUs the verify/copy-stream kernels (CRC, fp8 pack) may never occupy, so an
  // RCCL group kernel always finds free CUs to launch on instead of queueing
  // behind a burst of CRC launches that fills every CU's LDS (tools/contention).
  // -1: 32 when world > 1, 0 on one rank (no RCCL traffic). Ignored when verify_cus > 0.
  int reserve_cus = -1;
  // CUs of the verify stream, the last ones of the mask; RCCL and copies get the
  // rest (HipBackendConfig::verify_cus). -1: 32 (4 CUs on each XCD) with peers,
  // 128 when every landing is also unpacked (unpack_store), 0 (all CUs shared) alone.
  int verify_cus = -1;
  // RCCL communicator CTA (workgroup/channel) bounds via ncclCommInitRankConfig;
  // 0 keeps RCCL's own choice. More CTAs = more channels per P2P peer.
  int nccl_min_ctas = 0;
  int nccl_max_ctas = 0;
  bool nccl_register = false;  // register every HBM slot with the communicator (ncclCommRegister)
  // How the lane communicators are created: "parallel" = one ncclCommInitRankConfig
  // per lane from its own unique id, all inside one group (they initialize
  // concurrently), then every lane connected in one group; "split" = the world
  // communicator, then ncclCommSplit per lane one after another and a grouped
  // connect per ring distance (round 2's path; the bench's last fallback).
  std::string comm_init = "split";
};

// Comm lanes an engine of this config runs. 0 = auto: one lane per directed
// link (directed_lanes: 14 on 8 ranks) up to 8 ranks, else world-1 (at most 7)
// per-distance lanes; > 0: at most that many (per-distance scheme unless it
// equals directed_lanes).
inline int resolve_lanes(const PlannedConfig& c) {
  if (c.world <= 1) return 1;
  // several hosts: host-aware lanes while they stay few (a communicator and a
  // hardware queue each), else the per-distance lanes below
  if (c.lanes <= 0 && c.hosts > 1 && c.world % c.hosts == 0 && c.world / c.hosts <= 8 &&
      host_lanes(c.world, c.hosts, c.host_lane_classes) <= 32)
    return host_lanes(c.world, c.hosts, c.host_lane_classes);
  if (c.lanes <= 0) return c.world <= 8 ? directed_lanes(c.world) : std::min(c.world - 1, 7);
  return std::min(c.lanes, directed_lanes(c.world));
}

struct PlannedStats {
  int64_t bytes_sent = 0, bytes_recv = 0, bytes_staged = 0, bytes_verified = 0;
  int64_t groups = 0, pieces = 0, verify_failures = 0, unverified_pieces = 0;
  int64_t nacks = 0, injected = 0;
  int64_t suspects = 0, shrinks = 0, aborted_pieces = 0;  // elastic recovery
  double issue_ms = 0;  // host time spent enqueueing groups
  std::map<int, int64_t> peer_sent, peer_recv;  // bytes per peer rank (per-link counters)
  // device time of completed groups involving each peer / on each lane (ms)
  std::map<int, double> peer_busy_ms;
  std::map<int, double> peer_send_busy_ms;  // groups that sent to the peer (the directed link's own time)
  // groups that received from the peer: the same link timed at its other end.
  // A send's time includes waiting for its receive to be posted and a receive's
  // waiting for its send, so the closed loop takes the faster of the two ends
  // per link (Runtime.link_capacity): the later poster times the transfer alone.
  std::map<int, double> peer_recv_busy_ms;
  std::vector<double> lane_busy_ms;
  int lanes = 1;
  double comm_init_ms = 0, comm_connect_ms = 0;
  std::vector<double> lane_init_ms, lane_connect_ms;  // per comm lane (Backend::lane_init_ms)
  double comm_reform_ms = 0;  // last elastic re-form (abort + re-init after a shrink)
  int64_t paced = 0;  // issue attempts a token bucket deferred
  double disk_wait_ms = 0;  // time disk reads waited for the node-wide read budget
  // disk-tier bytes read with O_DIRECT (past every page cache of this OS) and
  // buffered (the filesystem refused O_DIRECT: they may come from memory)
  int64_t disk_direct_bytes = 0, disk_buffered_bytes = 0;
  int64_t order_violations = 0;  // sends that waited on a recv with a larger key (must stay 0)
  int64_t scratch_landings = 0;  // recvs of chunks already staged / resident here (landed in scratch)
  int64_t scratch_buffers = 0;   // scratch-landing buffers allocated (the pool grows only when all are busy)
  // device time the verify stream spent on checks (landing met -> check done):
  // against the session's wall time, the occupancy of the verify CUs
  double verify_busy_ms = 0;
  int64_t verify_calls = 0;   // Backend::verify calls (one event each; one launch per <= 16 chunks)
  int64_t verify_chunks = 0;  // chunk checks they carried (verify_chunks / verify_calls: the batching)
  // log2(us) histograms: bucket b counts latencies in [2^b, 2^(b+1)) us
  std::vector<int64_t> group_us_hist = std::vector<int64_t>(32, 0);  // P2P group issue -> complete
  std::vector<int64_t> land_us_hist = std::vector<int64_t>(32, 0);   // chunk issue -> landed + verified
};

// One op of an untimed link probe (PlannedEngine::probe).
struct ProbeOp {
  int peer = 0;          // partner rank
  bool send = true;
  int64_t bytes = 0;
  bool done = false;     // completed within the probe's time limit
  double ms = -1;        // device time of its group (lane reached it -> end); host time where unknown
  int lane = 0;
};

class PlannedEngine : public DataEngine {
 public:
  PlannedEngine(const PlannedConfig& cfg, std::unique_ptr<Backend> backend);
  ~PlannedEngine() override;

  // ---- setup (call while no session runs)
  uint8_t* provision(LayerID layer, int64_t size);
  uint8_t* device_ptr(LayerID layer);
  uint8_t* unpacked_ptr(LayerID layer);  // bf16 slot (unpack_store), nullptr if none yet
  void set_manifest(LayerID layer, const CrcManifest& m);
  void set_seeded(LayerID layer, bool device_resident);
  // The layer's host/disk source is already in the slot format (e.g. a layer
  // persisted by an earlier run): stage it byte for byte, without packing.
  void set_source_packed(LayerID layer, bool packed);
  // Grid chunks of a layer verified resident in HBM (call while no session runs).
  std::vector<int64_t> resident_chunks(LayerID layer);
  void reset_session();  // wait idle, forget landed chunks, poison non-seeded slots
  PlannedStats stats();
  std::string error();
  Backend* backend() { return backend_.get(); }
  // Untimed pre-flight probe between sessions: every op is posted at once, each
  // on its directed pair's lane (one group per lane), and timed; ops still
  // pending after timeout_s are returned with done = false (their lanes are
  // stalled: the buffers are then left allocated, a kernel may still use them).
  std::vector<ProbeOp> probe(const std::vector<ProbeOp>& ops, double timeout_s);

  // ---- DataEngine
  std::string name() const override { return backend_->name(); }
  Location target() const override { return Location::Device; }
  bool planned() const override { return true; }
  int64_t chunk_bytes() const override { return grid_; }  // chunk grid of HBM slots / transfers
  // Bytes a layer of `src_bytes` source bytes occupies in HBM and on the wire.
  int64_t slot_size(int64_t src_bytes) const;
  const PlannedConfig& config() const { return cfg_; }
  std::map<LayerID, CrcManifest> manifest() override;
  std::string new_comm_id() override { return backend_->new_comm_id(); }
  bool on_message(const MessagePtr& m) override;
  void send_range(NodeID dest, LayerID layer, int64_t offset, int64_t size, int64_t total, int64_t rate) override;
  void load_range(LayerID layer, int64_t offset, int64_t size, int64_t total, int64_t rate) override;
  void host_prefix_ready(LayerID layer, const uint8_t* base, int64_t prefix, int64_t total) override;
  void quiesce() override;
  void shutdown() override;
  int rank_of(NodeID n) const;

 private:
  enum class Kind : uint8_t { Send, Recv, Local };
  struct Piece {
    Kind kind;
    uint64_t seq;
    int64_t pidx;  // ordering key after the batch: the chunk index, or seq << 24 | chunk (job-major)
    int peer;      // rank
    LayerID layer;
    int64_t off, len, total;
    int64_t chunk;  // grid chunk index
    bool full;      // covers the whole grid chunk
    bool has_crc = false;
    uint32_t crc = 0;
    bool has_ccrc = false;  // partial piece: the CRC of its whole grid chunk
    uint32_t ccrc = 0;
    NodeID src_node = 0;
    bool bcast = false;  // collective from rank `peer` (root: Send with peer == own rank; others: Recv)
    int lane = 0;
    int64_t rate = 0;    // job pacing (B/s, 0 = unlimited)
    uint64_t batch = 0;  // add_batch ordinal (most significant part of the key)
    // A recv of a chunk this rank is already staging, or holds: it lands in this
    // scratch buffer instead of the live slot (issue_lane), so no byte of a
    // chunk is ever written by two copies at once.
    uint8_t* scratch = nullptr;
  };
  // Key: (batch, pidx, seq). Chunk-major batches (Message::order 0) set pidx to
  // the chunk index, job-major ones (order 1) to seq << 24 | chunk index.
  using Key = std::tuple<uint64_t, int64_t, uint64_t>;
  static Key key_of(const Piece& p) { return Key{p.batch, p.pidx, p.seq}; }
  struct PartChunk {
    RangeSet got;
    bool has_crc = false;
    uint32_t crc = 0;
  };
  struct Layer {
    int64_t size = 0;
    uint8_t* dev = nullptr;
    uint8_t* out = nullptr;          // unpack_store: bf16 slot (source size)
    bool seeded = false;
    CrcManifest manifest;
    const uint8_t* host = nullptr;   // host-tier source (set at first staging)
    std::string path;                // disk-tier source
    int64_t path_off = 0;
    bool src_packed = false;         // the source already holds the packed image (persisted layers)
    bool client_requested = false;   // ClientReq sent for this session
    int64_t stage_rate = -1;         // source tier LimitRate (-1: not looked up yet)
    int64_t host_prefix = -1;        // source bytes present at `host` (-1: all; a client stream still landing)
    int stage_tier = 0;
    std::vector<std::pair<int64_t, int64_t>> src_ranges;  // partial source: the byte ranges it holds
    bool ranges_known = false;       // src_ranges looked up this session
    // per chunk: 0 absent, 1 pending, 2 resident, 3 reading from disk,
    // 4 failed its CRC and awaits the leader's re-send (still forwardable: a
    // later receiver detects it and NACKs too)
    std::vector<uint8_t> st;
    std::vector<Ev> ev;              // staging event of a pending chunk (0: pending on the comm queue)
    std::vector<Key> rkey;           // key of the recv a pending chunk waits on (Key{}: staged)
    std::vector<uint8_t> want;       // inject Landed when resident (assigned here)
    std::vector<uint8_t> fails;      // CRC failures per chunk
    std::map<int64_t, PartChunk> part;  // chunks landing as several partial pieces
    std::map<int64_t, uint32_t> job_crc;  // CRCs from the leader's jobs (layers without a local manifest)
  };
  struct Verify {  // landing (recv group or staging copy) awaiting its check
    Ev ev = 0;
    double t0 = vclock::now();
    std::vector<Piece> pieces;
    std::vector<uint32_t> slots;  // CRC result slots, ~0u = not verified
  };
  struct PendingCheck {  // a landed or staged chunk whose check waits for the next flush_checks
    Piece piece;
    Ev wait = 0;                // its landing: a staging copy (held: ev_hold) or a P2P group / its corrupt mark
    bool held = false;
    uint32_t slot = ~0u;        // result slot, ~0u = not verified
    bool has_req = false;       // a check (plain or fused) to launch; else only the landing to wait for
    Backend::CheckReq req{};
    double t0 = vclock::now();
  };
  struct DiskRead {  // chunk of a disk-tier layer: pread into a bounce buffer, then H2D
    LayerID layer;
    int64_t chunk, file_off, len;
    std::string path;
    uint8_t* bounce = nullptr;
    bool ok = true;
  };
  struct ProbeJob {
    std::vector<ProbeOp> ops;
    double timeout_s = 0;
    bool finished = false;
  };
  struct Req {
    enum Type { Batch, Load, Reset, Stop, Shrink, HostReady, Probe } type;
    std::vector<XferJob> jobs;
    LayerID layer = 0;
    int64_t off = 0, len = 0;
    std::vector<NodeID> dead;  // Shrink
    uint64_t generation = 0;   // Shrink
    std::string comm_id;       // Shrink: the survivors' new communicator id
    const uint8_t* base = nullptr;  // HostReady: host copy; `off` = bytes present, `len` = total
    ProbeJob* probe = nullptr;  // Probe
    uint8_t order = 0;          // Batch: Message::order
  };
  void run_probe(ProbeJob& job);
  struct Inflight {  // a P2P group on a comm lane
    Ev ev;
    double t0;
    std::vector<int> peers;  // partner ranks
    std::vector<int> send_peers;  // ranks it sends to (point-to-point)
    std::vector<int> recv_peers;  // ranks it receives from (point-to-point)
  };
  struct Pace {  // token bucket, non-blocking (burst: one chunk; mode-3 jobs two, see pace_ready)
    double rate = 0, tokens = 0, burst = 0;
    double last = 0;
  };

  void run();
  void take_requests(bool block);
  void add_batch(std::vector<XferJob>& jobs, uint8_t order);
  bool issue_some();
  bool issue_lane(int lane);
  void poll();
  bool idle() const {
    for (auto& q : ops_)
      if (!q.empty()) return false;
    for (auto& q : inflight_)
      if (!q.empty()) return false;
    return verifies_.empty() && pending_checks_.empty() && disk_inflight_ == 0 && disk_wait_.empty() && local_wait_.empty() &&
           deferred_local_.empty() &&
           bounce_busy_.empty();
  }
  int lane_for(int peer, bool send) const {
    return send ? lane_of_hosts(cfg_.rank, peer, cfg_.world, lanes_, cfg_.hosts, cfg_.host_lane_classes)
                : lane_of_hosts(peer, cfg_.rank, cfg_.world, lanes_, cfg_.hosts, cfg_.host_lane_classes);
  }
  // Events shared by several chunks (a lane mark after a recv group): refcounted.
  void ev_hold(Ev e) {
    if (e) evref_[e]++;
  }
  void ev_drop(Ev e);
  void set_chunk_ev(Layer& L, int64_t c, Ev e);
  bool pace_ready(uint64_t key, int64_t rate, int64_t n);
  void pace_take(uint64_t key, int64_t rate, int64_t n);
  bool stage_paced(Layer& L, LayerID id, int64_t c);  // true: the tier's bucket defers this chunk
  // Elastic recovery: stop issuing, tell the leader which peers look dead, and
  // wait for its Shrink (or fail after group_timeout_s).
  // broken: the communicator failed (stop issuing) rather than merely stalled.
  void suspect(const std::vector<int>& peers, const std::string& why, bool broken);
  std::vector<int> inflight_peers() const;
  std::string describe_stall() const;
  void do_shrink(const std::vector<NodeID>& dead, uint64_t generation, const std::string& comm_id);
  void die();  // fault injection
  Layer& layer(LayerID id, int64_t size_hint = 0);
  // 1: resident or in flight on a device queue, 0: still reading from disk, -1: no source
  int ensure_chunk(Layer& L, LayerID id, int64_t c, bool want_landed);
  bool has_local_source(Layer& L, LayerID id, int64_t c);  // staging can supply chunk c
  bool source_covers(Layer& L, LayerID id, int64_t c);      // chunk c is not a hole of a partial source
  void stage_chunk(Layer& L, LayerID id, int64_t c);
  void stage_from(Layer& L, LayerID id, int64_t c, const uint8_t* src, uint8_t* bounce);
  void submit_disk(Layer& L, LayerID id, int64_t c);
  void pump_disk();
  void reader_loop();
  void landed(const Piece& p);
  // A partial recv piece landed: once the chunk's pieces cover it, queue its whole-chunk check to `out`.
  void partial_landed(Layer& L, const Piece& p, std::vector<Verify>& out);
  void nack(const Piece& p, Layer& L, uint32_t got);
  uint32_t crc_slot();
  // unpack_store: the fused check of chunk c (packed at L.dev) into its bf16 slot.
  Backend::CheckReq unpack_req(Layer& L, int64_t c, uint32_t slot);
  // Launch the pending checks as batched verifies (flush_checks), or forget them.
  void flush_checks();
  void drop_pending_checks();
  void fail(const std::string& what);
  int64_t src_len(const Layer& L, int64_t c) const;  // source bytes of chunk c
  int64_t src_grid(const Layer& L) const { return cfg_.pack == 1 && !L.src_packed ? cfg_.chunk_bytes : grid_; }

  PlannedConfig cfg_;
  int64_t grid_ = 0;  // chunk grid of HBM slots and transfers (packed chunk with pack=fp8)
  std::mt19937_64 inject_rng_;
  std::unique_ptr<Backend> backend_;
  NodeID self_node_ = 0;
  std::map<NodeID, int> node_rank_;
  uint32_t crc_next_ = 0;

  std::mutex req_mu_;
  CondVar req_cv_, idle_cv_;
  std::deque<Req> reqs_;
  bool busy_ = false;
  uint64_t resets_done_ = 0;

  // issue-thread state
  std::map<LayerID, Layer> layers_;
  int lanes_ = 1;
  std::vector<std::deque<Piece>> ops_;          // per lane, key order
  std::vector<std::deque<Inflight>> inflight_;  // per lane
  std::deque<Verify> verifies_;
  std::vector<PendingCheck> pending_checks_;  // checks not launched yet (staged and landed chunks)
  int pending_reqs_ = 0;                      // of them, chunk checks to launch
  std::vector<Ev> owned_waits_;               // landing events the engine releases after the flush
  std::vector<std::pair<LayerID, int64_t>> restage_;  // local chunks to stage again (bad CRC)
  std::deque<std::pair<LayerID, int64_t>> local_wait_;  // local promotions deferred by tier pacing
  std::deque<std::pair<LayerID, int64_t>> deferred_local_;  // promotions held back behind queued sends
  std::set<std::pair<LayerID, int64_t>> promoting_;  // of them, staged and not yet resident
  // keys of the queued (not yet posted) sends of each chunk: relay cuts, and
  // recvs of a chunk held back behind this rank's earlier-key send of it
  std::map<std::pair<LayerID, int64_t>, std::multiset<Key>> fwd_pending_;
  uint64_t batches_ = 0;
  std::map<Ev, int> evref_;
  std::map<uint64_t, Pace> pace_;
  bool recovering_ = false;  // issue thread: waiting for the leader's Shrink
  double recover_since_ = 0, last_suspect_ = -1e300;  // vclock::now() seconds
  int64_t groups_issued_ = 0;
  std::atomic<bool> dead_{false};  // fault injection: this rank "crashed"

  // disk tier: issue thread owns bounce_free_/disk_wait_; readers exchange via disk_mu_
  std::vector<uint8_t*> bounce_all_, bounce_free_;
  // Scratch landings (a recv of a chunk this rank stages or holds): chunk-sized
  // device buffers, reused and freed only at shutdown - a free mid-session
  // (hipFree synchronizes the device) hung a rank-death recovery whose
  // re-plan landed such chunks while its peers' RCCL kernels waited
  // (profiles/r6_insure).
  std::vector<uint8_t*> scratch_all_, scratch_free_;
  uint8_t* scratch_take();
  std::deque<std::pair<Ev, uint8_t*>> bounce_busy_;  // H2D copy event -> its bounce buffer
  std::deque<DiskRead> disk_wait_;                 // waiting for a bounce buffer
  std::mutex disk_mu_;
  CondVar disk_cv_;
  std::deque<DiskRead> disk_todo_, disk_done_;
  std::vector<std::thread> readers_;
  int disk_inflight_ = 0;
  std::unique_ptr<NodePacer> pacer_;  // node-shared disk budget (node_disk_rate > 0)

  std::mutex stats_mu_;
  PlannedStats stats_;
  std::string error_;
  std::atomic<bool> failed_{false};
  std::atomic<bool> stopped_{false};
  std::atomic<bool> stop_req_{false};
  std::thread th_;
  // Host-side watchdog: the issue thread marks every backend call that can
  // block inside RCCL/HIP; a monitor thread logs one that has not returned for
  // a few seconds (a hang there would also silence poll()'s group watchdog).
  struct CallMark {
    PlannedEngine* e;
    CallMark(PlannedEngine* eng, const char* what, int lane) : e(eng) {
      e->call_lane_ = lane;
      e->call_since_us_ = now_us();
      e->call_what_ = what;
    }
    ~CallMark() { e->call_what_ = nullptr; }
    static int64_t now_us() {
      return vclock::now_us();
    }
  };
  std::atomic<int64_t> loop_ticks_{0};  // issue-thread loop iterations (monitor: liveness)
  std::atomic<bool> idle_flag_{true};
  int64_t last_ticks_ = -1;             // monitor thread only
  bool stack_dumped_ = false;           // monitor thread only (DISSEM_STACK_DUMP)
  double ticks_since_ = vclock::now();
  int64_t completions_ = 0, quiet_mark_ = 0;  // completed groups; the count at the last progress check
  double quiet_since_ = vclock::now();
  std::atomic<const char*> call_what_{nullptr};
  std::atomic<int64_t> call_since_us_{0};
  std::atomic<int> call_lane_{0};
  std::thread monitor_;
  void monitor_loop();
};

constexpr uint32_t kCrcSlots = 1u << 16;
// Token-bucket keys (PlannedEngine::pace_ready): a mode-3 job, a rate-capped
// peer link, a source tier.
constexpr uint64_t kPaceJob = 1ull << 62, kPacePeer = 2ull << 62, kPaceTier = 3ull << 62;
// Chunks per verify launch (kern::kCrcBatchMax): at 64 MiB source chunks a
// batch of 16 is 1 GiB of bf16 per launch, where the fused kernel runs at
// its streaming rate; one chunk alone fills less than a round of the chip.
constexpr int kVerifyBatch = 16;
// Promotions (loads of a rank's own layers) staged ahead of the chunks its
// queued sends need: at most this many at a time (PlannedEngine::add_batch).
constexpr int kPromoteAhead = 2;

}  // namespace dissem
