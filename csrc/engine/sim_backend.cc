// Simulated device backend: host memory, in-order worker queues, and an
// in-process fabric with RCCL point-to-point matching semantics.
//
// The fabric matches the i-th send from rank A to rank B with the i-th recv on
// B from A (FIFO per lane and directed pair, like NCCL/RCCL P2P on one
// communicator). A group occupies its rank's lane queue until every op in it
// has been matched and copied, so a schedule that could deadlock on GPUs
// deadlocks here too; a bounded wait turns that into a reported failure
// instead of a hang.
//
// Timing model (SimTiming): a matched transfer occupies its directed link for
// len / link_bps after the link's previous transfer (full duplex, links
// independent); a staging copy occupies the rank's copy queue for
// len / stage_bps. With copy_bytes = false no payload moves (timing-only runs
// of full-size schedules in little memory). Multi-host fabrics (host, nic_bps)
// also charge a cross-host transfer to both ends' NICs.
//
// Every time here is vclock::now(): with the virtual clock on (core/vclock.h)
// the queues below wait in model time and a session's length is its modeled
// makespan, the same on every run and any host load; off, they sleep the
// modeled times on the wall clock.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <tuple>

#include "core/crc32c.h"
#include "core/fp8.h"
#include "core/queue.h"
#include "core/vclock.h"
#include "engine/backend.h"
#include "engine/planned_engine.h"

namespace dissem {

namespace {

struct SimEvent {
  std::atomic<int> state{0};  // 0 pending, 1 done, -1 failed
  double ms = -1;             // groups: time on the lane from dependencies met to completion
  std::mutex mu;
  CondVar cv;                 // state left 0 (queues waiting on it as a dependency)
  void set(int st) {
    {
      std::lock_guard<std::mutex> lk(mu);
      state = st;
    }
    cv.notify_all();
  }
};

struct Posted {
  uint8_t* ptr;
  int64_t len;
  bool done = false;
  bool bad = false;
  double done_at = 0;               // timing model: when the link finishes this transfer (vclock::now() s)
  double posted = vclock::now();
  double injected_s = 0;  // fault injection: this post came that late (SimTiming::recv_delay_s)
  double model_s = 0;     // modeled device time of the op (see Fabric::post)
};

struct Fabric {
  std::mutex mu;
  CondVar cv;
  bool aborted = false;  // a survivor shrank this communicator: every wait fails now
  // (lane, src, dst) -> sends, recvs
  std::map<std::tuple<int, int, int>, std::pair<std::deque<Posted*>, std::deque<Posted*>>> ch;
  SimFabricStats stats;
  std::set<int> crashed;  // fault injection: ranks whose posts no longer move bytes
  SimTiming timing;
  std::map<std::pair<int, int>, double> link_free;  // timing model: directed link busy until
  std::map<int, double> nic_out_free, nic_in_free;   // timing model: per-rank NIC busy until

  double link_rate(int src, int dst) const {
    auto it = timing.link.find({src, dst});
    return it != timing.link.end() ? it->second : timing.link_bps;
  }
  bool cross_host(int src, int dst) const {
    const auto& h = timing.host;
    return src < int(h.size()) && dst < int(h.size()) && h[size_t(src)] != h[size_t(dst)];
  }

  void post(int lane, int src, int dst, bool send, Posted* op) {
    std::lock_guard<std::mutex> lk(mu);
    if (aborted || crashed.count(send ? src : dst)) {  // aborted communicator / crashed poster: nothing moves
      op->done = op->bad = true;
      cv.notify_all();
      return;
    }
    auto& c = ch[{lane, src, dst}];
    (send ? c.first : c.second).push_back(op);
    while (!c.first.empty() && !c.second.empty()) {
      Posted* s = c.first.front();
      Posted* r = c.second.front();
      c.first.pop_front();
      c.second.pop_front();
      if (s->len != r->len) {
        s->bad = r->bad = true;
      } else {
        if (timing.copy_bytes) memcpy(r->ptr, s->ptr, size_t(s->len));
        stats.matched++;
        stats.bytes += s->len;
        double bps = link_rate(src, dst);
        const bool nic = timing.nic_bps > 0 && cross_host(src, dst);
        if (nic) bps = bps > 0 ? std::min(bps, timing.nic_bps) : timing.nic_bps;
        if (bps > 0) {
          // Each resource serves its transfers in match order: the directed
          // link, and across hosts the sender's NIC egress and the receiver's
          // NIC ingress as two queues of their own (a packet network keeps both
          // ends busy; a transfer waiting on one end never idles the other).
          // The transfer is done when its last queue is.
          // both ends posted: the transfer may start (timed from the posts
          // themselves, not from when this thread got the fabric's lock)
          const double now = std::max(s->posted, r->posted);
          const double dur = double(s->len) / bps;
          auto& free_at = link_free[{src, dst}];
          free_at = std::max(now, free_at) + dur;
          auto done = free_at;
          if (nic) {
            auto& o = nic_out_free[src];
            auto& i = nic_in_free[dst];
            o = std::max(now, o) + dur;
            i = std::max(now, i) + dur;
            done = std::max({done, o, i});
          }
          s->done_at = r->done_at = done;
          if (timing.trace) stats.transfers.emplace_back(src, dst, done - dur, done, s->len);
          // Modeled device time of each op: from the later of the two posts
          // (the transfer cannot start before both ends are there) to the end
          // on its link - queueing behind the link's earlier transfers
          // included - plus, for a send, any wait the fault injection put on
          // its receive. How late the simulator's own threads got to either
          // post never enters it, so rates derived from it (the closed loop's
          // busy throughput) are the same on an idle or a loaded host.
          const double span = done - std::max(s->posted, r->posted);
          s->model_s = span + r->injected_s;
          r->model_s = span;
        }
      }
      s->done = r->done = true;
    }
    cv.notify_all();
  }
  // Withdraw ops still queued (their group gave up): a later match must never
  // copy into or out of a buffer whose owner has moved on.
  void cancel(const std::vector<std::unique_ptr<Posted>>& ops) {
    std::lock_guard<std::mutex> lk(mu);
    for (auto& kv : ch)
      for (auto* q : {&kv.second.first, &kv.second.second})
        for (auto it = q->begin(); it != q->end();) {
          bool mine = false;
          for (auto& o : ops) mine = mine || o.get() == *it;
          it = mine ? q->erase(it) : std::next(it);
        }
  }
  // A crashed rank: withdraw every op it has posted and not yet matched (they
  // fail), so no peer copies into or out of its memory any more.
  void crash_rank(int rank) {
    std::lock_guard<std::mutex> lk(mu);
    crashed.insert(rank);  // ops its queues still post later fail at once
    for (auto& kv : ch) {
      const int src = std::get<1>(kv.first), dst = std::get<2>(kv.first);
      auto drop = [](std::deque<Posted*>& q) {
        for (auto* p : q) p->done = p->bad = true;
        q.clear();
      };
      if (src == rank) drop(kv.second.first);   // its sends
      if (dst == rank) drop(kv.second.second);  // its recvs
    }
    cv.notify_all();
  }
  // Returns false on timeout (deadlock) or a size mismatch.
  bool wait_all(const std::vector<std::unique_ptr<Posted>>& ops, double timeout_s) {
    std::unique_lock<std::mutex> lk(mu);
    bool ok = cv_wait_for(cv, lk, timeout_s, [&] {
      if (aborted) return true;
      for (auto& o : ops)
        if (!o->done) return false;
      return true;
    });
    if (!ok || aborted) return false;
    double until = 0;
    for (auto& o : ops) {
      if (o->bad) return false;
      until = std::max(until, o->done_at);
    }
    lk.unlock();
    vclock::sleep_until(until);  // the links are still moving these bytes
    return true;
  }
};

std::mutex g_fab_mu;
std::map<std::string, std::shared_ptr<Fabric>> g_fabrics;

// A shrunk communicator runs over the same links and hosts, its ranks
// renumbered without the dead ones: rank-indexed timing follows them.
SimTiming survivors_timing(const SimTiming& t, const std::vector<int>& dead, int old_world) {
  SimTiming out = t;
  std::vector<int> to(size_t(old_world), -1);
  for (int r = 0, k = 0; r < old_world; ++r)
    if (std::find(dead.begin(), dead.end(), r) == dead.end()) to[size_t(r)] = k++;
  if (!t.host.empty()) {
    out.host.clear();
    for (int r = 0; r < old_world && r < int(t.host.size()); ++r)
      if (to[size_t(r)] >= 0) out.host.push_back(t.host[size_t(r)]);
  }
  out.link.clear();
  for (auto& kv : t.link) {
    const int a = kv.first.first, b = kv.first.second;
    if (a < old_world && b < old_world && to[size_t(a)] >= 0 && to[size_t(b)] >= 0)
      out.link[{to[size_t(a)], to[size_t(b)]}] = kv.second;
  }
  return out;
}

std::shared_ptr<Fabric> fabric(const std::string& key, const Fabric* inherit = nullptr,
                               const std::vector<int>& dead = {}, int old_world = 0) {
  std::lock_guard<std::mutex> lk(g_fab_mu);
  auto& f = g_fabrics[key];
  if (!f) {
    f = std::make_shared<Fabric>();
    if (inherit) f->timing = survivors_timing(inherit->timing, dead, old_world);
  }
  return f;
}

class Queue {
 public:
  Queue() : th_(vclock::spawn([this] { loop(); }, "sim-queue")) {}
  ~Queue() { stop(); }
  void push(std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(fn));
    }
    cv_.notify_all();
  }
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return q_.empty() && !running_; });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) return;
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty() || stop_; });
        if (q_.empty()) return;
        fn = std::move(q_.front());
        q_.pop_front();
        running_ = true;
      }
      fn();
      {
        std::lock_guard<std::mutex> lk(mu_);
        running_ = false;
      }
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  CondVar cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false, running_ = false;
  std::thread th_;
};

bool wait_event(const std::shared_ptr<SimEvent>& e, double timeout_s) {
  std::unique_lock<std::mutex> lk(e->mu);
  e->cv.wait_for_s(lk, timeout_s, [&] { return e->state.load() != 0; });
  return e->state.load() > 0;
}

class SimBackend : public Backend {
 public:
  SimBackend(const std::string& key, int rank, int world, int lanes)
      : key_(key), rank_(rank), world_(world), fab_(fabric(key)), results_(kCrcSlots, 0) {
    for (int l = 0; l < std::max(1, lanes); ++l) comm_.push_back(std::make_unique<Queue>());
  }
  ~SimBackend() override { destroy(false); }
  std::string name() const override { return "sim"; }
  int lanes() const override { return int(comm_.size()); }

  uint8_t* alloc(int64_t n) override {
    auto* p = new uint8_t[size_t(std::max<int64_t>(n, 1))]();
    return p;
  }
  void free(uint8_t* p) override { delete[] p; }
  uint8_t* alloc_host(int64_t n) override {
    void* p = nullptr;
    if (posix_memalign(&p, 4096, size_t(std::max<int64_t>(n, 4096)))) throw std::bad_alloc();
    return static_cast<uint8_t*>(p);
  }
  void free_host(uint8_t* p) override { ::free(p); }
  void zero_sync(uint8_t* p, int64_t n) override {
    sync_all();
    memset(p, 0, size_t(n));
  }

  // Staging occupies the copy queue for n / stage_bps (timing model).
  void stage_delay(double t0, int64_t n) {
    const double bps = fab_->timing.stage_bps;
    if (bps <= 0) return;
    if (fab_->timing.trace) {
      std::lock_guard<std::mutex> lk(fab_->mu);
      fab_->stats.stages.emplace_back(rank_, t0, t0 + double(n) / bps, n);
    }
    vclock::sleep_until(t0 + double(n) / bps);
  }

  Ev stage(uint8_t* dst, const uint8_t* src, int64_t n) override {
    auto [id, ev] = make_event();
    const bool copy = fab_->timing.copy_bytes;
    copy_.push([=] {
      const double t0 = vclock::now();
      if (copy) memcpy(dst, src, size_t(n));
      stage_delay(t0, n);
      ev->set(1);
    });
    return id;
  }

  Ev stage_pack(uint8_t* dst, const uint8_t* src, int64_t n_src, int block) override {
    auto [id, ev] = make_event();
    const bool copy = fab_->timing.copy_bytes;
    copy_.push([=] {
      const double t0 = vclock::now();
      const int64_t n = n_src / 2;
      if (copy) fp8::pack_host(reinterpret_cast<const uint16_t*>(src), n, dst, reinterpret_cast<float*>(dst + n), block);
      stage_delay(t0, n_src);
      ev->set(1);
    });
    return id;
  }

  Ev corrupt(uint8_t* p, int lane) override {
    auto [id, ev] = make_event();
    lane_q(lane).push([=] {
      const uint32_t pat = 0xA5A5A5A5u;
      memcpy(p, &pat, 4);
      ev->set(1);
    });
    return id;
  }

  Ev mark(int lane) override {
    auto [id, ev] = make_event();
    lane_q(lane).push([=] { ev->set(1); });
    return id;
  }

  Ev group(const std::vector<XOp>& ops, const std::vector<Ev>& waits, int lane) override {
    auto [id, ev] = make_event();
    std::vector<std::shared_ptr<SimEvent>> deps;
    for (Ev w : waits) deps.push_back(lookup(w));
    int rank = rank_;
    auto fab = fab_;
    lane_q(lane).push([=] {
      for (size_t i = 0; i < deps.size(); ++i) {
        auto& d = deps[i];
        if (!d || !wait_event(d, fab->timing.wait_s)) {
          set_error(std::string("group dependency failed: event ") + std::to_string(waits[i]) +
                    (d ? (d->state.load() < 0 ? " failed" : " timed out") : " was already released"));
          ev->set(-1);
          return;
        }
      }
      double injected = 0;
      if (auto rd = fab->timing.recv_delay_s.find(rank); rd != fab->timing.recv_delay_s.end() && rd->second > 0)
        for (auto& o : ops)
          if (!o.send && !o.bcast) {
            vclock::sleep_for(rd->second);
            injected = rd->second;
            break;
          }
      auto mk = [&](const XOp& o) {
        auto p = std::make_unique<Posted>(Posted{o.ptr, o.len});
        if (!o.send) p->injected_s = injected;
        return p;
      };
      std::vector<std::unique_ptr<Posted>> posted;
      // Optional RCCL round model: ops grouped by ring distance, each round
      // waits for the previous one (collectives stay in round 0).
      std::vector<std::vector<XOp>> rounds(1);
      if (fab->timing.p2p_rounds) {
        rounds.assign(size_t(std::max(1, world_)), {});
        for (auto& o : ops) {
          int d = 0;
          if (!o.bcast) d = o.send ? (o.peer - rank + world_) % world_ : (rank - o.peer + world_) % world_;
          rounds[size_t(d)].push_back(o);
        }
      } else {
        rounds[0] = ops;
      }
      for (auto& round : rounds) {
      if (round.empty()) continue;
      const size_t first = posted.size();
      for (auto& o : round) {
        if (o.bcast) {
          // Broadcast = the root sends to every other rank, each of which receives
          // from the root: same matching (and deadlock) semantics as a collective.
          if (o.peer == rank) {
            for (int r = 0; r < world_; ++r)
              if (r != rank) {
                posted.push_back(mk(o));
                fab->post(lane, rank, r, true, posted.back().get());
              }
          } else {
            posted.push_back(mk(o));
            fab->post(lane, o.peer, rank, false, posted.back().get());
          }
          continue;
        }
        if (o.peer < 0 || o.peer >= world_ || o.peer == rank) {
          set_error("bad peer");
          ev->set(-1);
          return;
        }
        posted.push_back(mk(o));
        if (o.send) fab->post(lane, rank, o.peer, true, posted.back().get());
        else fab->post(lane, o.peer, rank, false, posted.back().get());
      }
      if (rounds.size() > 1) {
        std::vector<std::unique_ptr<Posted>> cur;
        for (size_t i = first; i < posted.size(); ++i) cur.push_back(std::move(posted[i]));
        posted.resize(first);
        const bool ok = fab->wait_all(cur, fab->timing.wait_s);
        for (auto& c : cur) posted.push_back(std::move(c));
        if (!ok) break;
      }
      }
      if (!fab->wait_all(posted, fab->timing.wait_s)) {
        fab->cancel(posted);
        set_error("P2P group did not complete (deadlock or size mismatch)");
        ev->set(-1);
        return;
      }
      // The group's device time: its longest op in the model (ops of one group
      // run concurrently; with the timing model off, transfers take no time).
      double ms = 0;
      for (auto& p : posted) ms = std::max(ms, p->model_s * 1e3);
      ev->ms = ms;
      ev->set(1);
    });
    return id;
  }

  double group_ms(Ev e) override {
    auto ev = lookup(e);
    return ev && ev->state.load() > 0 ? ev->ms : -1;
  }

  Ev verify(const std::vector<CheckReq>& reqs, const std::vector<Ev>& waits) override {
    auto [id, ev] = make_event();
    std::vector<std::shared_ptr<SimEvent>> deps;
    for (Ev w : waits)
      if (w) deps.push_back(lookup(w));
    const bool copy = fab_->timing.copy_bytes;
    verify_.push([=] {
      for (auto& d : deps)
        if (!d || !wait_event(d, fab_->timing.wait_s)) {
          ev->set(-1);
          return;
        }
      const SimTiming& tm = fab_->timing;
      if (tm.verify_bps > 0 || tm.verify_launch_s > 0) {
        int64_t bytes = 0;
        for (const CheckReq& r : reqs) bytes += r.out ? fp8::packed_len(r.n, r.block) : r.n;
        const double dur = tm.verify_launch_s + (tm.verify_bps > 0 ? double(bytes) / tm.verify_bps : 0.0);
        const double t0 = vclock::now();
        vclock::sleep_until(t0 + dur);
        ev->ms = dur * 1e3;
      }
      for (const CheckReq& r : reqs) {
        if (r.n <= 0) continue;
        if (!copy) {  // timing-only run: no bytes moved, the check is charged above and passes
          results_[r.slot] = r.expect;
          continue;
        }
        if (!r.out) {
          results_[r.slot] = crc32c(r.p, size_t(r.n));
          continue;
        }
        const int64_t n = r.n / 2;  // fp8 values of the chunk
        results_[r.slot] = crc32c(r.p, size_t(fp8::packed_len(r.n, r.block)));
        if (copy)
          fp8::unpack_host(r.p, reinterpret_cast<const float*>(r.p + n), n, reinterpret_cast<uint16_t*>(r.out), r.block);
      }
      ev->set(1);
    });
    return id;
  }

  int query(Ev e) override {
    auto ev = lookup(e);
    if (!ev) return -1;
    return ev->state.load();
  }
  void release(Ev e) override {
    std::lock_guard<std::mutex> lk(ev_mu_);
    events_.erase(e);
  }
  uint32_t crc_result(uint32_t slot) override { return results_[slot]; }
  std::string async_error() override {
    std::lock_guard<std::mutex> lk(ev_mu_);
    return error_;
  }
  int shrink(const std::vector<int>& dead, uint64_t generation, const std::string&) override {
    {
      std::lock_guard<std::mutex> lk(fab_->mu);
      fab_->aborted = true;  // like NCCL_SHRINK_ABORT: in-flight groups fail now
    }
    fab_->cv.notify_all();
    sync_all();
    int new_rank = 0;
    for (int r = 0; r < rank_; ++r)
      if (std::find(dead.begin(), dead.end(), r) == dead.end()) ++new_rank;
    const int old_world = world_;
    world_ -= int(dead.size());
    rank_ = new_rank;
    {
      std::lock_guard<std::mutex> lk(ev_mu_);
      error_.clear();
    }
    fab_ = fabric(key_ + "/shrink" + std::to_string(generation), fab_.get(), dead, old_world);
    return rank_;
  }

  void crash() override { fab_->crash_rank(rank_); }

  void sync_all() override {
    for (auto& q : comm_) q->drain();
    copy_.drain();
    verify_.drain();
  }
  void destroy(bool) override {
    for (auto& q : comm_) q->stop();
    copy_.stop();
    verify_.stop();
  }

 private:
  std::pair<Ev, std::shared_ptr<SimEvent>> make_event() {
    auto e = std::make_shared<SimEvent>();
    std::lock_guard<std::mutex> lk(ev_mu_);
    Ev id = ++next_;
    events_[id] = e;
    return {id, e};
  }
  Queue& lane_q(int lane) { return *comm_.at(fab_->timing.serialize_lanes ? 0 : size_t(lane)); }
  std::shared_ptr<SimEvent> lookup(Ev e) {
    if (!e) return nullptr;
    std::lock_guard<std::mutex> lk(ev_mu_);
    auto it = events_.find(e);
    return it == events_.end() ? nullptr : it->second;
  }
  void set_error(const std::string& s) {
    std::lock_guard<std::mutex> lk(ev_mu_);
    if (error_.empty()) error_ = s;
  }

  std::string key_;
  int rank_, world_;
  std::shared_ptr<Fabric> fab_;
  std::vector<uint32_t> results_;
  std::mutex ev_mu_;
  std::map<Ev, std::shared_ptr<SimEvent>> events_;
  Ev next_ = 0;
  std::string error_;
  std::vector<std::unique_ptr<Queue>> comm_;
  Queue copy_, verify_;
};

}  // namespace

std::unique_ptr<Backend> make_sim_backend(const std::string& comm_key, int rank, int world, int lanes) {
  return std::make_unique<SimBackend>(comm_key, rank, world, lanes);
}

void sim_set_timing(const std::string& comm_key, const SimTiming& t) {
  auto f = fabric(comm_key);
  std::lock_guard<std::mutex> lk(f->mu);
  f->timing = t;
  f->link_free.clear();
}

void sim_clear_trace(const std::string& comm_key) {
  auto f = fabric(comm_key);
  std::lock_guard<std::mutex> lk(f->mu);
  f->stats.transfers.clear();
  f->stats.stages.clear();
}

SimFabricStats sim_fabric_stats(const std::string& comm_key) {
  auto f = fabric(comm_key);
  std::lock_guard<std::mutex> lk(f->mu);
  return f->stats;
}

}  // namespace dissem
