// Device backend of the planned data engine. The engine (csrc/engine/
// planned_engine.cc) owns scheduling: piece order, group formation, chunk
// states, verification bookkeeping, pacing. A backend owns the device: memory,
// the ordered queues and completion events:
//   * `lanes()` comm lanes - each an independent communicator + in-order queue
//     for grouped P2P (a directed pair a->b always uses lane_of(a, b), on both
//     ends), so a peer that is slow to post stalls only its own lane;
//   * copy queue(s) for host->device staging;
//   * a verify queue for CRC checks.
//
//  * HipBackend (csrc/gpu/hip_backend.cc): HBM via hipMalloc, RCCL grouped
//    P2P over xGMI (one communicator + stream per lane), hipMemcpyAsync H2D
//    staging, the gfx950 CRC32C kernel, hipEvents.
//  * SimBackend (csrc/engine/sim_backend.cc): host memory, worker threads as
//    in-order queues, and an in-process "fabric" that matches sends and recvs
//    between ranks FIFO per (lane, src, dst) exactly like RCCL P2P (a group
//    blocks its lane until every op in it is matched). Optional timing model:
//    per directed link bandwidth and per-rank staging bandwidth. Used to test
//    multi-rank schedules, deadlock freedom and timing without GPUs.
#pragma once

#include <algorithm>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

namespace dissem {

using Ev = uint64_t;  // 0 = no event

struct XOp {
  bool send;
  int peer;  // partner rank; the root rank when bcast
  uint8_t* ptr;
  int64_t len;
  bool bcast = false;  // collective broadcast of [ptr, ptr+len) from rank `peer` to every rank (in place)
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  virtual void init_thread() {}  // called on the engine's issue thread
  virtual uint8_t* alloc(int64_t n) = 0;
  virtual void free(uint8_t* p) = 0;
  virtual void zero_sync(uint8_t* p, int64_t n) = 0;
  // page-aligned host staging memory the copy queue can DMA from (pinned on GPUs)
  virtual uint8_t* alloc_host(int64_t n) = 0;
  virtual void free_host(uint8_t* p) = 0;
  // copy queue: async host -> device copy; event fires when it landed
  virtual Ev stage(uint8_t* dst, const uint8_t* src_host, int64_t n) = 0;
  // copy queue: host -> device copy of `n_src` bytes of bf16, then fp8-pack them
  // into dst in the packed chunk layout of core/fp8.h
  virtual Ev stage_pack(uint8_t* dst, const uint8_t* src_host, int64_t n_src, int block) = 0;
  // Independent comm lanes (>= 1).
  virtual int lanes() const { return 1; }
  // comm lane `lane`: wait for `waits`, then one grouped set of P2P sends/recvs
  virtual Ev group(const std::vector<XOp>& ops, const std::vector<Ev>& waits, int lane = 0) = 0;
  // An event that fires once everything queued so far on comm lane `lane` is done.
  virtual Ev mark(int lane) = 0;
  // Device time (ms) of a completed group, from the moment its lane reached it
  // (waits satisfied) to its end; < 0 if unknown.
  virtual double group_ms(Ev e) {
    (void)e;
    return -1;
  }
  // comm lane (fault injection): overwrite 4 bytes at p behind everything
  // queued so far on the lane, e.g. a chunk a group just received
  virtual Ev corrupt(uint8_t* p, int lane = 0) = 0;
  // verify queue: wait for `waits`, then check every request - all of them in
  // one event (one launch per kCrcBatchMax requests on GPUs, the fold inside
  // it): the CRC32C of [p, p+n) into result slot `slot`. A request with `out`
  // is an fp8-packed chunk (core/fp8.h layout of `n` bf16 SOURCE bytes with
  // `block`-element scales): its packed bytes are checked and dequantized to
  // `out` in the same pass (the fused kernel). No requests: an ordering
  // marker on the verify queue.
  struct CheckReq {
    const uint8_t* p;
    int64_t n;
    uint32_t slot;
    uint8_t* out = nullptr;
    int block = 0;
    // The CRC the engine expects. Only the timing-only simulator uses it
    // (SimTiming::copy_bytes false moves no bytes, so it reports this value).
    uint32_t expect = 0;
  };
  virtual Ev verify(const std::vector<CheckReq>& reqs, const std::vector<Ev>& waits) = 0;
  virtual int query(Ev e) = 0;  // 1 done, 0 pending, -1 failed
  virtual void release(Ev e) = 0;
  virtual uint32_t crc_result(uint32_t slot) = 0;
  virtual std::string async_error() { return ""; }
  // Elastic recovery: abort every in-flight comm-queue operation, then continue
  // on a communicator of the surviving ranks (the same call on every survivor,
  // with the same `dead` ranks, `generation` and `comm_id`). Returns this
  // rank's new index. RCCL: ncclCommAbort, then ncclCommInitRank of the
  // survivors with the leader's fresh unique id (comm_id).
  virtual std::string new_comm_id() { return ""; }
  virtual int shrink(const std::vector<int>& dead, uint64_t generation, const std::string& comm_id) {
    (void)dead;
    (void)generation;
    (void)comm_id;
    throw std::runtime_error(name() + " backend cannot shrink its communicator");
  }
  virtual void sync_all() = 0;
  virtual void destroy(bool abort) = 0;
  // Fault injection: this rank "crashes" - nothing it posted may still move
  // bytes (a dead process's outstanding ops vanish with it).
  virtual void crash() {}
  virtual double comm_init_ms() const { return 0; }     // communicator set-up, connects included
  virtual double comm_connect_ms() const { return 0; }  // the connect part
  // Per lane: its communicator's set-up (split: that lane's ncclCommSplit, lane
  // 0 the world init; parallel: every lane = the one concurrent group) and its
  // share of the connects (per distance it serves; one value for all when the
  // connects run as one group).
  virtual std::vector<double> lane_init_ms() const { return {}; }
  virtual std::vector<double> lane_connect_ms() const { return {}; }
};

// Lanes. Every directed pair (src -> dst) has one lane, computed identically
// on both ends. Two schemes:
//  * per distance (lanes <= world-1): lane = (d - 1) % lanes with d the ring
//    distance dst - src; with world-1 lanes each lane of a rank carries one
//    send peer (rank+d) and one recv peer (rank-d), one RCCL round each;
//  * per directed link (lanes == directed_lanes(world), the default on up to 8
//    ranks): the links of distance d form cycles r -> r+d -> ...; each link's
//    lane is (d, color of its sender in a proper coloring of its cycle), so a
//    rank's send to rank+d and its recv from rank-d sit on different lanes and
//    every directed xGMI link progresses on its own - no lockstep along the
//    ring. Cycles of even length need 2 colors, odd ones 3.
inline int lane_gcd(int a, int b) { return b ? lane_gcd(b, a % b) : a; }
inline int lane_colors(int world) {
  for (int d = 1; d < world; ++d)
    if ((world / lane_gcd(world, d)) % 2) return 3;
  return 2;
}
inline int directed_lanes(int world) { return world > 1 ? (world - 1) * lane_colors(world) : 1; }
inline int lane_color(int src, int d, int world, int colors) {
  const int g = lane_gcd(world, d), len = world / g;
  int k = 0;  // position of src on its cycle r0, r0+d, r0+2d, ...
  for (int x = src % g; x != src; x = (x + d) % world) ++k;
  if (colors == 3 && len % 2 == 1 && k == len - 1) return 2;
  return k % 2;
}
inline int lane_of(int src, int dst, int world, int lanes) {
  if (lanes <= 1 || world <= 1) return 0;
  const int d = ((dst - src) % world + world) % world;  // 1 .. world-1
  if (lanes == directed_lanes(world)) {
    const int c = lane_colors(world);
    return (d - 1) * c + lane_color(((src % world) + world) % world, d, world, c);
  }
  return (d - 1) % lanes;
}

// Several hosts (multi-node): `hosts` hosts of g = world / hosts ranks each,
// rank r on host r / g (torchrun's rank order). A pair on one host uses the
// directed lanes of a host's xGMI mesh (by local index). A pair across hosts
// uses a lane of its (host distance, local distance class, sender color):
// the cycle coloring over hosts keeps a GPU's sends to and recvs from another
// host on different lanes, and `classes` (1..g) spreads a GPU's remote peers
// over that many lanes per direction (classes = g: one lane per directed link,
// = directed_lanes(world) lanes in all; fewer classes share a lane between
// remote peers, which then wait on each other in key order).
// classes <= 0: auto, as many as fit 32 lanes in all (2 hosts x 8 GPUs: 8
// classes = one lane per directed link, 30 lanes; 3-4 hosts: 3 classes). The
// 2 x 8-GPU sim (profiles/r3_multihost/): mode 1 runs about as fast with 4
// classes (22 lanes) as with 8, 2x slower with 1 (16 lanes); the three-level
// mode-0 broadcast 663 ms with 8 classes vs 880-920 with 4.
inline int host_lane_classes(int world, int hosts, int classes) {
  const int g = world / hosts;
  if (classes <= 0) classes = (32 - directed_lanes(g)) / ((hosts - 1) * lane_colors(hosts));
  return std::max(1, std::min(classes, g));
}
inline int host_lanes(int world, int hosts, int classes) {
  if (hosts <= 1 || world % hosts) return directed_lanes(world);
  const int g = world / hosts, k = host_lane_classes(world, hosts, classes);
  return directed_lanes(g) + (hosts - 1) * k * lane_colors(hosts);
}
inline int lane_of_hosts(int src, int dst, int world, int lanes, int hosts, int classes) {
  if (hosts <= 1 || world % hosts || lanes != host_lanes(world, hosts, classes)) return lane_of(src, dst, world, lanes);
  const int g = world / hosts, hs = src / g, hd = dst / g, k = host_lane_classes(world, hosts, classes);
  if (hs == hd) return lane_of(src % g, dst % g, g, directed_lanes(g));
  const int dh = ((hd - hs) % hosts + hosts) % hosts, c = lane_colors(hosts);
  const int dl = ((dst % g - src % g) % g + g) % g;
  return directed_lanes(g) + ((dh - 1) * k + dl % k) * c + lane_color(hs, dh, hosts, c);
}

struct SimFabricStats {
  int64_t matched = 0, bytes = 0;
  // SimTiming::trace: every timed transfer as (src, dst, start s, end s, bytes)
  std::vector<std::tuple<int, int, double, double, int64_t>> transfers;
  std::vector<std::tuple<int, double, double, int64_t>> stages;  // (rank, start s, end s, bytes)
};

// Timing model of the simulated fabric (all rates in bytes/s, 0 = instant).
struct SimTiming {
  double link_bps = 0;                            // every directed rank->rank link
  std::map<std::pair<int, int>, double> link;     // per directed link override
  double stage_bps = 0;                           // host->device staging per rank (PCIe)
  bool copy_bytes = true;                         // false: move no payload bytes (timing-only runs)
  // Model RCCL's P2P schedule with few channels: a group's ops run in rounds of
  // one ring distance each (send to rank+d, recv from rank-d), round d+1 only
  // after round d completed. Irregular groups can then deadlock where
  // independent ops would not; one-distance groups (lanes = world-1) cannot.
  bool p2p_rounds = false;
  // Several hosts (multi-node runs): rank -> host id (empty: one host). A
  // transfer between ranks on different hosts also occupies the sender's NIC
  // (egress) and the receiver's NIC (ingress), each nic_bps per direction, at
  // min(link, NIC): one NIC per GPU, shared by all of that GPU's remote peers.
  std::vector<int> host;
  double nic_bps = 0;
  // A group not complete after this many seconds counts as deadlocked. Timed
  // runs of congested schedules can queue a transfer behind longer than the
  // default (the link and NIC reservations are FIFO).
  double wait_s = 30;
  // Fault injection: a rank that posts every P2P group holding a receive this
  // many seconds late (its peers' sends wait for it, as an RCCL send waits
  // for the matching receive): the closed loop must not read that as slow links.
  std::map<int, double> recv_delay_s;
  // Fault injection for the schedule tests: every comm lane of a rank runs on
  // ONE queue (its groups one after another, as if the lanes were one stream).
  // The model-time upper bounds in tests/test_timing_sim.py must catch it.
  bool serialize_lanes = false;
  // The verify queue's device time: every launch costs verify_launch_s plus
  // its bytes (packed bytes read; the fused unpack's bf16 writes are not
  // charged) at verify_bps - the measured CRC walk on the verify stream's CUs
  // (profiles/r5_walk: ~1 TB/s on 32 CUs, ~24 us for a lone 64 MiB chunk on
  // all). 0 = instant, as before.
  double verify_bps = 0;
  double verify_launch_s = 0;
  // Record every timed transfer and staging copy (sim_fabric_trace): the
  // per-link timelines that show where a schedule leaves links idle.
  bool trace = false;
};

// In-process simulated fabric: ranks of one "communicator" share `comm_key`.
std::unique_ptr<Backend> make_sim_backend(const std::string& comm_key, int rank, int world, int lanes = 1);
SimFabricStats sim_fabric_stats(const std::string& comm_key);
void sim_clear_trace(const std::string& comm_key);
// Set the timing model of a fabric (before its ranks start moving bytes).
void sim_set_timing(const std::string& comm_key, const SimTiming& t);

}  // namespace dissem
