#include "gpu/hip_backend.h"

#include <hip/hip_runtime_api.h>
#include <rccl.h>

#include <chrono>
#include <algorithm>
#include <cstring>
#include <thread>
#include <map>
#include <mutex>
#include <vector>

#include "core/log.h"
#include "kernels/kernels.h"

namespace dissem {

namespace {

#define HIP_OK(expr)                                                                                        \
  do {                                                                                                      \
    hipError_t _e = (expr);                                                                                 \
    if (_e != hipSuccess) throw std::runtime_error(std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

#define NCCL_OK(expr)                                                                                         \
  do {                                                                                                        \
    ncclResult_t _r = (expr);                                                                                 \
    if (_r != ncclSuccess) throw std::runtime_error(std::string(#expr " failed: ") + ncclGetErrorString(_r)); \
  } while (0)

class HipBackend : public Backend {
 public:
  explicit HipBackend(const HipBackendConfig& cfg) : cfg_(cfg) {
    HIP_OK(hipSetDevice(cfg_.device));
    const int lanes = std::max(1, cfg_.lanes);
    // One in-order stream per comm lane. With several lanes each must sit on a
    // hardware queue of its own: two lanes sharing one would run their RCCL
    // kernels in submission order, and a kernel waiting for a peer would hold
    // back the other lane's kernel that peer may itself be waiting for. A
    // CU-masked stream gets a dedicated queue, so extra lanes are created with
    // a mask of every CU (profiles/: Queue_Id per lane).
    const int part = std::max(0, cfg_.verify_cus);  // CUs kept for the verify stream alone
    for (int l = 0; l < lanes; ++l) {
      hipStream_t s = nullptr;
      if (lanes > 1 || part > 0) {
        s = create_stream_reserving(cfg_.device, part, /*dedicated=*/true);
      } else {
        HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      }
      comm_.push_back(s);
    }
    nccl_.assign(size_t(lanes), nullptr);
    const int keep_free = part > 0 ? part : cfg_.reserve_cus;  // CUs the copy streams stay off
    copy_ = create_stream_reserving(cfg_.device, keep_free);
    // Two SDMA copy queues in alternation keep the PCIe link busier across copy
    // boundaries (h2dbench: 56.8 -> 57.4 GB/s; bench 56.0 -> 56.9 GB/s). With
    // RCCL in the process only when the copy queues are CU-masked: a masked
    // stream gets a hardware queue of its own, so no copy can end up queued
    // behind a comm-stream kernel that waits for a peer.
    if ((cfg_.world == 1 && !cfg_.self_comm) || keep_free > 0)
      copy2_ = create_stream_reserving(cfg_.device, keep_free);
    verify_ = part > 0 ? create_stream_on_last(cfg_.device, part) : create_stream_reserving(cfg_.device, cfg_.reserve_cus);
    // The verify kernels size the last round of their grid for the CUs the
    // verify stream may use (kernels.h `cus`).
    {
      int cus = 0;
      HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg_.device));
      verify_cus_ = part > 0 ? std::min(part, cus)
                    : cfg_.reserve_cus > 0 && cfg_.reserve_cus < cus ? cus - cfg_.reserve_cus : 0;
    }
    // The fold words of one verify launch ({acc, count} per item): zeroed once,
    // every launch leaves them zeroed (kernels.h).
    HIP_OK(hipMalloc(&ws_, kern::crc32c_batch_workspace_bytes()));
    HIP_OK(hipMemsetAsync(ws_, 0, kern::crc32c_batch_workspace_bytes(), verify_));
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&crc_host_), kCrcSlots * sizeof(uint32_t),
                         hipHostMallocMapped | hipHostMallocCoherent));
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&crc_dev_), crc_host_, 0));
    // CRC tables before any RCCL traffic
    HIP_OK(kern::crc32c_warm(verify_));
    HIP_OK(hipStreamSynchronize(verify_));
    if (cfg_.world > 1 || cfg_.self_comm) {
      std::string ids = cfg_.nccl_uid;
      if (cfg_.world == 1 && ids.empty()) ids = nccl_unique_id(int(nccl_.size()));
      init_comm(ids);
    }
  }

  ncclConfig_t comm_config() const {
    ncclConfig_t nc = NCCL_CONFIG_INITIALIZER;
    if (cfg_.nccl_min_ctas > 0) nc.minCTAs = cfg_.nccl_min_ctas;
    if (cfg_.nccl_max_ctas > 0) nc.maxCTAs = cfg_.nccl_max_ctas;
    return nc;
  }

  // `ids`: one ncclUniqueId per lane (parallel init), or a single id (split).
  void init_comm(const std::string& ids) {
    const size_t n = nccl_.size(), idb = sizeof(ncclUniqueId);
    if (ids.size() != idb && ids.size() != n * idb)
      throw std::runtime_error("nccl_uid must hold 1 or " + std::to_string(n) + " ncclUniqueIds");
    const bool parallel = cfg_.parallel_init && ids.size() == n * idb;
    auto t0 = log::now_us();
    std::vector<ncclConfig_t> ncs(n, comm_config());
    lane_init_ms_.assign(n, 0.0);
    lane_connect_ms_.assign(n, 0.0);
    if (parallel) {
      // Every lane communicator from its own unique id, all in one group: RCCL
      // runs the inits (bootstrap, topology, channel set-up) concurrently.
      // Measured at 8 ranks sharing one GPU it was slower than split
      // (profiles/r3_init2: 18.7-19.1 s vs 16.3-17.1 s), so split is the
      // default; each lane records the group's time.
      std::vector<ncclUniqueId> uid(n);
      memcpy(uid.data(), ids.data(), n * idb);
      NCCL_OK(ncclGroupStart());
      for (size_t l = 0; l < n; ++l) NCCL_OK(ncclCommInitRankConfig(&nccl_[l], cfg_.world, uid[l], cfg_.rank, &ncs[l]));
      NCCL_OK(ncclGroupEnd());
      std::fill(lane_init_ms_.begin(), lane_init_ms_.end(), double(log::now_us() - t0) / 1e3);
    } else {
      ncclUniqueId id;
      memcpy(&id, ids.data(), idb);
      NCCL_OK(ncclCommInitRankConfig(&nccl_[0], cfg_.world, id, cfg_.rank, &ncs[0]));
      lane_init_ms_[0] = double(log::now_us() - t0) / 1e3;
      // Further lanes: independent communicators over the same ranks (own
      // channels and connections; collective split, same order on every rank).
      for (size_t l = 1; l < n; ++l) {
        const auto ts = log::now_us();
        ncs[l].splitShare = 0;
        NCCL_OK(ncclCommSplit(nccl_[0], 0, cfg_.rank, &nccl_[l], &ncs[l]));
        lane_init_ms_[l] = double(log::now_us() - ts) / 1e3;
      }
    }
    const auto t1 = log::now_us();
    connect_all(parallel);
    init_ms_ = double(log::now_us() - t0) / 1e3;
    connect_ms_ = double(log::now_us() - t1) / 1e3;
    log::info(cfg_.rank).i("world", cfg_.world).i("lanes", int64_t(n)).s("init", parallel ? "parallel" : "split")
        .f("init_ms", init_ms_).f("connect_ms", connect_ms_).msg("rccl communicators ready");
  }

  // RCCL connects a pair lazily inside the first ncclGroupEnd that uses it, and
  // that call blocks the host thread until the peer runs the same setup. With
  // several lanes, ranks reach their first groups on different lanes in
  // different orders (mode 2's dynamic jobs), and two ranks each blocked in a
  // setup the other has not reached yet would hang. So every lane connects
  // every distance it serves (and lane 0 its broadcast ring) here, in one fixed
  // order on every rank.
  //
  // `one_group`: every distance in a single group across the lane
  // communicators (the same fixed order on every rank, so the per-lane
  // connection set-ups RCCL runs inside ncclGroupEnd cannot wait on each other
  // in a cycle: the lowest lane some rank waits on has all of its ranks there);
  // otherwise one group per distance (round 2).
  void connect_all(bool one_group = false) {
    const int world = cfg_.world, lanes = int(nccl_.size());
    if (world < 2) return;
    if (!probe_) HIP_OK(hipMalloc(&probe_, 64 * 1024));
    uint8_t* sbuf = static_cast<uint8_t*>(probe_);
    if (one_group) NCCL_OK(ncclGroupStart());
    for (int d = 1; d < world; ++d) {
      const int to = (cfg_.rank + d) % world, from = (cfg_.rank - d + world) % world;
      const size_t ls = size_t(lane_of_hosts(cfg_.rank, to, world, lanes, cfg_.hosts, cfg_.host_lane_classes)),
                   lr = size_t(lane_of_hosts(from, cfg_.rank, world, lanes, cfg_.hosts, cfg_.host_lane_classes));
      uint8_t* rbuf = sbuf + 4096 * size_t(std::min(d, 15));  // distinct landing per recv of the group
      const auto tc = log::now_us();
      if (!one_group) NCCL_OK(ncclGroupStart());
      NCCL_OK(ncclSend(sbuf, 64, ncclUint8, to, nccl_[ls], comm_[ls]));
      NCCL_OK(ncclRecv(rbuf, 64, ncclUint8, from, nccl_[lr], comm_[lr]));
      if (!one_group) {
        NCCL_OK(ncclGroupEnd());
        const double ms = double(log::now_us() - tc) / 1e3;  // the distance's send + recv set-up
        if (ls < lane_connect_ms_.size()) lane_connect_ms_[ls] += ms / 2;
        if (lr < lane_connect_ms_.size()) lane_connect_ms_[lr] += ms / 2;
      }
    }
    if (one_group) {
      const auto tc = log::now_us();
      NCCL_OK(ncclGroupEnd());
      std::fill(lane_connect_ms_.begin(), lane_connect_ms_.end(), double(log::now_us() - tc) / 1e3);
    }
    NCCL_OK(ncclBroadcast(sbuf, sbuf, 64, ncclUint8, 0, nccl_[0], comm_[0]));
    for (hipStream_t s : comm_) HIP_OK(hipStreamSynchronize(s));
  }
  ~HipBackend() override { destroy(false); }
  std::string name() const override { return "rccl"; }
  int lanes() const override { return int(comm_.size()); }
  double comm_init_ms() const override { return init_ms_; }
  double comm_connect_ms() const override { return connect_ms_; }
  std::vector<double> lane_init_ms() const override { return lane_init_ms_; }
  std::vector<double> lane_connect_ms() const override { return lane_connect_ms_; }

  void init_thread() override { HIP_OK(hipSetDevice(cfg_.device)); }

  // Layer slots are allocated once per session set-up; with nccl_register each
  // is also registered with the communicator (ncclCommRegister), which lets
  // RCCL use the user buffer directly where its transport supports it.
  void register_slot(uint8_t* p, int64_t n) {
    if (!cfg_.nccl_register || !nccl_[0]) return;
    std::vector<void*> hs;
    for (auto c : nccl_) {
      void* h = nullptr;
      ncclResult_t r = ncclCommRegister(c, p, size_t(n), &h);
      if (r != ncclSuccess) {
        log::warn(cfg_.rank).s("error", ncclGetErrorString(r)).msg("ncclCommRegister failed; slot stays unregistered");
        h = nullptr;
      }
      hs.push_back(h);
    }
    regs_[p] = {n, hs};
  }
  void deregister_slot(uint8_t* p) {
    auto it = regs_.find(p);
    if (it == regs_.end()) return;
    for (size_t l = 0; l < it->second.second.size() && l < nccl_.size(); ++l)
      if (nccl_[l] && it->second.second[l]) (void)ncclCommDeregister(nccl_[l], it->second.second[l]);
    regs_.erase(it);
  }

  uint8_t* alloc(int64_t n) override {
    HIP_OK(hipSetDevice(cfg_.device));
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, size_t(std::max<int64_t>(n, 1))));
    register_slot(static_cast<uint8_t*>(p), std::max<int64_t>(n, 1));
    return static_cast<uint8_t*>(p);
  }
  void free(uint8_t* p) override {
    deregister_slot(p);
    (void)hipFree(p);
  }
  uint8_t* alloc_host(int64_t n) override {
    void* p = nullptr;
    HIP_OK(hipHostMalloc(&p, size_t(std::max<int64_t>(n, 4096)), hipHostMallocDefault));
    return static_cast<uint8_t*>(p);
  }
  void free_host(uint8_t* p) override { (void)hipHostFree(p); }
  void zero_sync(uint8_t* p, int64_t n) override {
    // On the copy queue, never a comm lane: a lane may still hold an RCCL
    // kernel waiting for a dead peer after a failed session.
    HIP_OK(hipMemsetAsync(p, 0, size_t(n), copy_));
    HIP_OK(hipStreamSynchronize(copy_));
  }

  Ev stage(uint8_t* dst, const uint8_t* src, int64_t n) override {
    hipStream_t s = copy2_ && (flip_ ^= true) ? copy2_ : copy_;
    HIP_OK(hipMemcpyAsync(dst, src, size_t(n), hipMemcpyHostToDevice, s));
    return record(s);
  }

  Ev stage_pack(uint8_t* dst, const uint8_t* src, int64_t n_src, int block) override {
    // bf16 lands in a device scratch chunk, then the gfx950 pack kernel writes
    // the packed chunk into the layer slot. One scratch per copy queue: both
    // steps are ordered on that queue, and packing (~22 us per 64 MiB) is
    // noise next to the PCIe copy (~1.2 ms).
    const int q = copy2_ && (flip_ ^= true) ? 1 : 0;
    hipStream_t s = q ? copy2_ : copy_;
    if (n_src > scratch_bytes_[q]) {
      // Sized for a whole source chunk on first use, so it never grows in a
      // session: hipFree synchronizes the device, comm lanes included.
      HIP_OK(hipStreamSynchronize(s));
      if (scratch_[q]) HIP_OK(hipFree(scratch_[q]));
      scratch_[q] = nullptr;
      const int64_t want = std::max(n_src, cfg_.max_chunk_bytes);
      HIP_OK(hipMalloc(&scratch_[q], size_t(want)));
      scratch_bytes_[q] = want;
    }
    HIP_OK(hipMemcpyAsync(scratch_[q], src, size_t(n_src), hipMemcpyHostToDevice, s));
    const int64_t n = n_src / 2;
    HIP_OK(kern::fp8_pack(static_cast<const uint16_t*>(scratch_[q]), n, dst, reinterpret_cast<float*>(dst + n), block,
                          s));
    return record(s);
  }

  Ev corrupt(uint8_t* p, int lane) override {
    hipStream_t s = comm_.at(size_t(lane));
    HIP_OK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p), 0xA5A5A5A5u, 1, s));
    return record(s);
  }

  Ev mark(int lane) override { return record(comm_.at(size_t(lane))); }

  Ev group(const std::vector<XOp>& ops, const std::vector<Ev>& waits, int lane) override {
    hipStream_t s = comm_.at(size_t(lane));
    ncclComm_t c = nccl_.at(size_t(lane));
    for (Ev w : waits) HIP_OK(hipStreamWaitEvent(s, ev(w), 0));
    // Timed group: a timing event where the lane reaches the group (its waits
    // met) and one at its end; group_ms() reads the device time between them.
    hipEvent_t start = timed();
    HIP_OK(hipEventRecord(start, s));
    if (!ops.empty()) {
      if (!c) throw std::runtime_error("P2P group on a single-rank engine");
      NCCL_OK(ncclGroupStart());
      for (auto& o : ops) {
        if (o.bcast) NCCL_OK(ncclBroadcast(o.ptr, o.ptr, size_t(o.len), ncclUint8, o.peer, c, s));
        else if (o.send) NCCL_OK(ncclSend(o.ptr, size_t(o.len), ncclUint8, o.peer, c, s));
        else NCCL_OK(ncclRecv(o.ptr, size_t(o.len), ncclUint8, o.peer, c, s));
      }
      NCCL_OK(ncclGroupEnd());
    }
    hipEvent_t end = timed();
    HIP_OK(hipEventRecord(end, s));
    const Ev e = reinterpret_cast<Ev>(end);
    starts_[e] = start;
    return e;
  }

  double group_ms(Ev e) override {
    auto it = starts_.find(e);
    if (it == starts_.end()) return -1;
    float ms = 0;
    return hipEventElapsedTime(&ms, it->second, ev(e)) == hipSuccess ? double(ms) : -1;
  }

  // Verify work is timed like a group (group_ms): from where the verify
  // stream reaches it (its landings met) to its end - the engine sums that into
  // verify_busy_ms, the verify CUs' occupancy. Plain checks and fused
  // check+unpacks go out as batched launches of up to kCrcBatchMax chunks
  // each (a 64 MiB chunk alone fills less than one round of the chip).
  Ev verify(const std::vector<CheckReq>& reqs, const std::vector<Ev>& waits) override {
    for (Ev w : waits)
      if (w) HIP_OK(hipStreamWaitEvent(verify_, ev(w), 0));
    hipEvent_t start = timed();
    HIP_OK(hipEventRecord(start, verify_));
    std::vector<kern::CrcItem> plain;
    std::vector<kern::FusedItem> fused;
    int block = 0;
    auto flush_plain = [&] {
      if (!plain.empty()) HIP_OK(kern::crc32c_batch(plain.data(), int(plain.size()), ws_, verify_, verify_cus_));
      plain.clear();
    };
    auto flush_fused = [&] {
      if (!fused.empty())
        HIP_OK(kern::fp8_verify_unpack_batch(fused.data(), int(fused.size()), block, ws_, verify_, verify_cus_));
      fused.clear();
    };
    for (const CheckReq& r : reqs) {
      if (r.n <= 0) continue;
      if (r.out) {
        if (block && r.block != block) flush_fused();
        block = r.block;
        fused.push_back(kern::FusedItem{r.p, r.n, reinterpret_cast<uint16_t*>(r.out), crc_dev_ + r.slot});
        if (fused.size() == size_t(kern::kCrcBatchMax)) flush_fused();
      } else {
        plain.push_back(kern::CrcItem{r.p, r.n, crc_dev_ + r.slot});
        if (plain.size() == size_t(kern::kCrcBatchMax)) flush_plain();
      }
    }
    flush_fused();
    flush_plain();
    return timed_end(verify_, start);
  }

  int query(Ev e) override {
    hipError_t r = hipEventQuery(ev(e));
    if (r == hipSuccess) return 1;
    if (r == hipErrorNotReady) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    if (err_.empty()) err_ = hipGetErrorString(r);
    return -1;
  }
  void release(Ev e) override {
    if (!e) return;
    auto it = starts_.find(e);
    if (it != starts_.end()) {
      timed_pool_.push_back(it->second);
      timed_pool_.push_back(ev(e));
      starts_.erase(it);
      return;
    }
    pool_.push_back(ev(e));
  }
  uint32_t crc_result(uint32_t slot) override { return __atomic_load_n(&crc_host_[slot], __ATOMIC_ACQUIRE); }
  std::string async_error() override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!err_.empty()) return err_;
    }
    for (auto c : nccl_) {
      if (!c) continue;
      ncclResult_t ar = ncclSuccess;
      if (ncclCommGetAsyncError(c, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress)
        return ncclGetErrorString(ar);
    }
    return "";
  }
  // The survivors' communicators after a shrink: one id per lane (parallel init).
  std::string new_comm_id() override { return nccl_unique_id(cfg_.parallel_init ? int(nccl_.size()) : 1); }

  int shrink(const std::vector<int>& dead, uint64_t, const std::string& comm_id) override {
    if (!nccl_[0]) throw std::runtime_error("shrink without a communicator");
    if (comm_id.empty() || comm_id.size() % sizeof(ncclUniqueId)) throw std::runtime_error("shrink: bad communicator id");
    // Abort first: P2P groups waiting on the dead rank are terminated, so the
    // comm streams drain. (ncclCommShrink would keep the bootstrap, but the RCCL
    // PyTorch loads into the process predates it; abort + re-init of the
    // survivors works with any RCCL.)
    abort_all();
    log::warn(cfg_.rank).i("lanes", int64_t(nccl_.size())).msg("rccl communicators aborted; draining queues");
    std::vector<std::pair<uint8_t*, int64_t>> regd;  // re-register with the new communicators
    for (auto& kv : regs_) regd.push_back({kv.first, kv.second.first});
    regs_.clear();
    int new_rank = 0;
    for (int r = 0; r < cfg_.rank; ++r)
      if (std::find(dead.begin(), dead.end(), r) == dead.end()) ++new_rank;
    cfg_.world -= int(dead.size());
    cfg_.hosts = 1;  // the survivors no longer fill whole hosts (as the engine's lane map)
    cfg_.rank = new_rank;
    {
      std::lock_guard<std::mutex> lk(mu_);
      err_.clear();
    }
    // Bounded drain of every queue (an aborted kernel must have exited).
    std::vector<hipStream_t> all(comm_);
    for (hipStream_t s : {copy_, verify_, copy2_}) all.push_back(s);
    for (hipStream_t s : all) {
      if (!s) continue;
      hipEvent_t e;
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      HIP_OK(hipEventRecord(e, s));
      auto t0 = std::chrono::steady_clock::now();
      hipError_t q;
      while ((q = hipEventQuery(e)) == hipErrorNotReady) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20)) {
          (void)hipEventDestroy(e);
          throw std::runtime_error("queues did not drain after ncclCommShrink");
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      (void)hipEventDestroy(e);
    }
    init_comm(comm_id);
    for (auto& pr : regd) register_slot(pr.first, pr.second);
    return new_rank;
  }

  // Abort every lane's communicator at once, one thread each. ncclCommAbort
  // raises the comm's abort flag and then waits for its work to drain; a lane
  // kernel of another, not yet aborted communicator that waits for a dead peer
  // would never drain, so aborting the lanes one after another can hang. In
  // parallel every flag is up within microseconds and every kernel exits.
  void abort_all() {
    std::vector<std::thread> ths;
    for (auto& c : nccl_) {
      if (!c) continue;
      ncclComm_t comm = c;
      c = nullptr;
      ths.emplace_back([comm] { (void)ncclCommAbort(comm); });
    }
    for (auto& t : ths) t.join();
  }

  void sync_all() override {
    (void)hipSetDevice(cfg_.device);
    for (hipStream_t s : comm_) (void)hipStreamSynchronize(s);
    (void)hipStreamSynchronize(copy_);
    if (copy2_) (void)hipStreamSynchronize(copy2_);
    (void)hipStreamSynchronize(verify_);
  }
  void destroy(bool abort) override {
    if (destroyed_) return;
    destroyed_ = true;
    (void)hipSetDevice(cfg_.device);
    if (!abort) sync_all();
    if (abort) {
      abort_all();
    } else {
      for (size_t l = nccl_.size(); l-- > 0;) {  // split lanes before the parent
        if (nccl_[l]) ncclCommDestroy(nccl_[l]);
        nccl_[l] = nullptr;
      }
    }
    for (auto e : pool_) (void)hipEventDestroy(e);
    pool_.clear();
    for (auto& kv : starts_) {
      timed_pool_.push_back(kv.second);
      timed_pool_.push_back(ev(kv.first));
    }
    starts_.clear();
    for (auto e : timed_pool_) (void)hipEventDestroy(e);
    timed_pool_.clear();
    if (ws_) (void)hipFree(ws_);
    if (probe_) (void)hipFree(probe_);
    for (void* p : scratch_)
      if (p) (void)hipFree(p);
    if (crc_host_) (void)hipHostFree(crc_host_);
    for (hipStream_t s : comm_) (void)hipStreamDestroy(s);
    (void)hipStreamDestroy(copy_);
    if (copy2_) (void)hipStreamDestroy(copy2_);
    (void)hipStreamDestroy(verify_);
  }

 private:
  static hipEvent_t ev(Ev e) { return reinterpret_cast<hipEvent_t>(e); }
  Ev record(hipStream_t s) {
    hipEvent_t e;
    if (!pool_.empty()) {
      e = pool_.back();
      pool_.pop_back();
    } else {
      HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    HIP_OK(hipEventRecord(e, s));
    return reinterpret_cast<Ev>(e);
  }
  Ev timed_end(hipStream_t s, hipEvent_t start) {
    hipEvent_t end = timed();
    HIP_OK(hipEventRecord(end, s));
    const Ev e = reinterpret_cast<Ev>(end);
    starts_[e] = start;
    return e;
  }
  hipEvent_t timed() {
    hipEvent_t e;
    if (!timed_pool_.empty()) {
      e = timed_pool_.back();
      timed_pool_.pop_back();
    } else {
      HIP_OK(hipEventCreate(&e));
    }
    return e;
  }

  HipBackendConfig cfg_;
  std::vector<hipStream_t> comm_;  // one per lane
  hipStream_t copy_ = nullptr, verify_ = nullptr;
  hipStream_t copy2_ = nullptr;  // second H2D queue
  std::map<uint8_t*, std::pair<int64_t, std::vector<void*>>> regs_;  // registered slots: size, handle per lane
  bool flip_ = false;
  std::vector<ncclComm_t> nccl_;  // one per lane (lane 0: the world communicator, others split from it)
  double init_ms_ = 0, connect_ms_ = 0;
  std::vector<double> lane_init_ms_, lane_connect_ms_;
  void* probe_ = nullptr;  // connect_all() scratch
  std::map<Ev, hipEvent_t> starts_;  // timed group end -> its start event
  std::vector<hipEvent_t> timed_pool_;
  void* ws_ = nullptr;  // fold words of the verify launches
  int verify_cus_ = 0;  // CUs of the verify stream (0 = all): kernels.h `cus`
  void* scratch_[2] = {nullptr, nullptr};  // bf16 landing chunk for stage_pack, per copy queue
  int64_t scratch_bytes_[2] = {0, 0};
  uint32_t* crc_host_ = nullptr;
  uint32_t* crc_dev_ = nullptr;
  std::vector<hipEvent_t> pool_;  // issue-thread only
  std::mutex mu_;
  std::string err_;
  bool destroyed_ = false;
};

}  // namespace

std::unique_ptr<Backend> make_hip_backend(const HipBackendConfig& cfg) { return std::make_unique<HipBackend>(cfg); }

hipStream_t create_stream_reserving(int device, int reserve, bool dedicated) {
  HIP_OK(hipSetDevice(device));
  hipStream_t s = nullptr;
  int cus = 0;
  HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  if (reserve >= cus) reserve = 0;
  if (reserve <= 0 && !dedicated) {
    HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
  }
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0u);
  for (int cu = 0; cu < cus - reserve; ++cu) mask[size_t(cu / 32)] |= 1u << (cu % 32);
  HIP_OK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  return s;
}

hipStream_t create_stream_on_last(int device, int n) {
  HIP_OK(hipSetDevice(device));
  int cus = 0;
  HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  n = std::max(1, std::min(n, cus));
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0u);
  for (int cu = cus - n; cu < cus; ++cu) mask[size_t(cu / 32)] |= 1u << (cu % 32);
  hipStream_t s = nullptr;
  HIP_OK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  return s;
}

std::shared_ptr<HostBuffer> alloc_pinned(int64_t size) {
  void* p = nullptr;
  HIP_OK(hipHostMalloc(&p, size_t(std::max<int64_t>(size, 1)), hipHostMallocDefault));
  return HostBuffer::wrap(static_cast<uint8_t*>(p), size,
                          std::shared_ptr<void>(p, [](void* q) { (void)hipHostFree(q); }));
}

std::string nccl_unique_id(int count) {
  std::string out;
  for (int i = 0; i < std::max(1, count); ++i) {
    ncclUniqueId id;
    NCCL_OK(ncclGetUniqueId(&id));
    out.append(reinterpret_cast<const char*>(&id), sizeof id);
  }
  return out;
}

}  // namespace dissem
