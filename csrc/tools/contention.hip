// contention: does a burst of verify kernels delay an RCCL-like kernel launched
// on another stream, and does reserving CUs on the verify stream fix it?
//
//   bin/contention [-trials N] [-reserve R]
//
// In the planned engine a P2P group lands up to 7 chunks at once; their CRC
// (one batched launch; one 144 KiB-LDS workgroup per CU) runs on the verify
// stream while the next RCCL group kernel waits to launch on the comm stream.
// The probe here stands in for that kernel: 28 workgroups x 256 threads, 16 KiB
// of LDS each, ~20 us of work. For each trial we enqueue the batched CRC of 7
// 64 MiB chunks on the verify stream, then the probe, and time the probe from
// its enqueue to its end (HIP events on its own idle stream), and the burst.
// Verify stream without a CU mask vs one created with R CUs left free, with
// the CRC grid at 256 workgroups or capped at the stream's 256 - R CUs.
//
// Bandwidth, not only launch delay: a 32-workgroup HBM -> HBM copy (16 B per
// lane, grid-stride; the stand-in for one comm lane's RCCL P2P kernel moving a
// chunk) on an all-CU dedicated queue, alone and while batched CRC bursts run
// back to back on the verify stream (unmasked / masked with R CUs free). The
// copy's GB/s (bytes copied per second) says whether the CU reservation leaves
// a lane its bandwidth: 7 lanes at >= 60 GB/s each need >= 420 GB/s.
//
// Continuous verification at the landing rate (-paced): at N = 8 a GPU lands
// 7 links x ~64 GB/s = ~450 GB/s, every byte CRC-checked. For 10 s a host
// thread enqueues one batched CRC of 7 x 64 MiB chunks every 7 x 64 MiB /
// 450 GB/s (~1 ms) on the verify stream with the grid capped at C workgroups,
// while a 64-workgroup copy runs back to back on a comm-lane-like queue. Per
// cap: the copy's GB/s against its alone rate, and whether the verify kept up
// (the batches still pending at the end and the time to drain them).
#include <atomic>
#include <chrono>
#include <thread>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <map>
#include <set>
#include <vector>

#include <rccl/rccl.h>

#include "kernels/kernels.h"

#define CHECK(x)                                                       \
  do {                                                                 \
    hipError_t err_ = (x);                                             \
    if (err_ != hipSuccess) {                                          \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(err_)); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

__global__ void __launch_bounds__(256) probe_kernel(uint32_t* out, uint64_t ticks) {
  __shared__ uint32_t lds[4096];  // 16 KiB, like a comm kernel's staging space
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
  uint32_t acc = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) acc += lds[(acc + threadIdx.x) & 4095];
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                  int64_t n16) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += int64_t(gridDim.x) * 256) dst[i] = src[i];
}

static hipStream_t make_stream(int reserve, bool dedicated = false) {
  hipStream_t s = nullptr;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (reserve <= 0 && !dedicated) {
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
  }
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0u);
  for (int cu = 0; cu < cus - reserve; ++cu) mask[size_t(cu / 32)] |= 1u << (cu % 32);
  CHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  return s;
}

int paced(double secs, double land_gbps, const std::vector<int>& caps);

// A stream on the CUs whose mask bit `pick(cu)` says (every CU's bit set or not).
template <class Pick>
static hipStream_t make_masked(Pick pick) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint32_t> mask(size_t((cus + 31) / 32), 0u);
  for (int cu = 0; cu < cus; ++cu)
    if (pick(cu, cus)) mask[size_t(cu / 32)] |= 1u << (cu % 32);
  hipStream_t s = nullptr;
  CHECK(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  return s;
}

// Which XCD (HW_REG_XCC_ID) and which CU inside it (HW_REG_HW_ID) each
// workgroup of a long kernel ran on: the map from CU-mask bits to the
// hardware that the verify partition relies on. Measured (profiles/r4_contention/
// cumap.jsonl): bit i is CU i / 8 of XCD i mod 8, workgroups go to the XCDs
// round-robin whatever the mask, and an XCD left without a CU runs its share on
// all of its CUs.
__global__ void __launch_bounds__(64) where_kernel(uint32_t* __restrict__ out, int64_t spin) {
  const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID[15:0]
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  int64_t t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

static int cumap() {
  CHECK(hipSetDevice(0));
  const int blocks = 2048;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&out, size_t(blocks) * 2 * sizeof(uint32_t)));
  std::vector<uint32_t> h(size_t(blocks) * 2);
  struct Mask {
    const char* name;
    int every, phase, n;  // every < 0: contiguous last n; every == 0: contiguous first n
  };
  const Mask masks[] = {{"all", 1, 0, 0}, {"last32", -1, 0, 32}, {"first32", 0, 0, 32}, {"every8th", 8, 7, 32},
                        {"bits_224_255_complement", -2, 0, 32}};
  for (const Mask& m : masks) {
    hipStream_t st = make_masked([m](int cu, int cus) {
      if (m.every == 1) return true;
      if (m.every == -1) return cu >= cus - m.n;
      if (m.every == -2) return cu < cus - m.n;
      if (m.every == 0) return cu < m.n;
      return cu % m.every == m.phase;
    });
    CHECK(hipMemsetAsync(out, 0xff, size_t(blocks) * 2 * sizeof(uint32_t), st));
    where_kernel<<<blocks, 64, 0, st>>>(out, 200000);
    CHECK(hipStreamSynchronize(st));
    CHECK(hipMemcpy(h.data(), out, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::map<uint32_t, int> per_xcc;
    std::map<uint32_t, std::set<uint32_t>> cus_of_xcc;
    for (int b = 0; b < blocks; ++b) {
      const uint32_t x = h[size_t(2 * b)] & 0xf, hw = h[size_t(2 * b + 1)];
      ++per_xcc[x];
      // gfx9 HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]
      cus_of_xcc[x].insert(((hw >> 13) & 7) * 32 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15));
    }
    printf("{\"case\": \"cumap\", \"mask\": \"%s\", \"workgroups_per_xcd\": {", m.name);
    bool first = true;
    for (auto& [x, c] : per_xcc) {
      printf("%s\"%u\": %d", first ? "" : ", ", x, c);
      first = false;
    }
    printf("}, \"distinct_cus_per_xcd\": {");
    first = true;
    for (auto& [x, c] : cus_of_xcc) {
      printf("%s\"%u\": %zu", first ? "" : ", ", x, c.size());
      first = false;
    }
    printf("}}\n");
    fflush(stdout);
    CHECK(hipStreamDestroy(st));
  }
  CHECK(hipFree(out));
  return 0;
}

// ---- RCCL's own P2P kernel beside continuous verification (-rccl SECS): a
// one-rank communicator sends 256 MiB to itself and receives it (one group
// per transfer, back to back on the lane stream), timed per group, alone and
// beside verification paced at the landing rate: unmasked full grid, grid
// capped at 32, and partitioned (verify on the last 32 CU-mask bits, the lane
// on the rest - the engine's layout with peers).
#define NCHECK(x)                                                                       \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

static int rccl_paced(double secs, double land_gbps) {
  CHECK(hipSetDevice(0));
  ncclUniqueId id;
  NCHECK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  NCHECK(ncclCommInitRank(&comm, 1, id, 0));
  const int64_t chunk = 64ll << 20, nchunks = 7, xfer = 256ll << 20;
  uint8_t *buf = nullptr, *sbuf = nullptr, *rbuf = nullptr;
  CHECK(hipMalloc(&buf, size_t(chunk * nchunks)));
  CHECK(dissem::kern::fill_random(buf, chunk * nchunks, 42, nullptr));
  CHECK(hipMalloc(&sbuf, size_t(xfer)));
  CHECK(hipMalloc(&rbuf, size_t(xfer)));
  CHECK(hipMemset(sbuf, 3, size_t(xfer)));
  const int kRing = 64;
  const size_t wsb = dissem::kern::crc32c_batch_workspace_bytes();
  uint8_t* ws = nullptr;
  CHECK(hipMalloc(&ws, wsb * kRing));
  CHECK(hipMemset(ws, 0, wsb * kRing));  // fold words: zeroed once (kernels.h)
  uint32_t* crc = nullptr;
  CHECK(hipMalloc(&crc, size_t(kRing) * nchunks * sizeof(uint32_t)));
  const double period_s = double(chunk * nchunks) / (land_gbps * 1e9);
  auto pct = [](std::vector<float> v, double q) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.f : v[size_t(q * double(v.size() - 1))];
  };
  auto rccl_run = [&](hipStream_t lane, double dur, std::vector<float>& gbps) {
    const int n = 16;
    std::vector<hipEvent_t> ev(size_t(n) + 1);
    for (auto& e : ev) CHECK(hipEventCreate(&e));
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(dur);
    while (std::chrono::steady_clock::now() < t_end) {
      CHECK(hipEventRecord(ev[0], lane));
      for (int k = 0; k < n; ++k) {
        NCHECK(ncclGroupStart());
        NCHECK(ncclSend(sbuf, size_t(xfer), ncclChar, 0, comm, lane));
        NCHECK(ncclRecv(rbuf, size_t(xfer), ncclChar, 0, comm, lane));
        NCHECK(ncclGroupEnd());
        CHECK(hipEventRecord(ev[size_t(k) + 1], lane));
      }
      CHECK(hipStreamSynchronize(lane));
      for (int k = 0; k < n; ++k) {
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, ev[size_t(k)], ev[size_t(k) + 1]));
        gbps.push_back(float(double(xfer) / (double(ms) * 1e-3) / 1e9));
      }
    }
    for (auto& e : ev) CHECK(hipEventDestroy(e));
  };
  // warm: RCCL connections, CRC tables
  hipStream_t lane_all = make_stream(0, true);
  {
    std::vector<float> w;
    rccl_run(lane_all, 0.2, w);
    hipStream_t v0;
    CHECK(hipStreamCreateWithFlags(&v0, hipStreamNonBlocking));
    dissem::kern::CrcItem it[nchunks];
    for (int64_t c = 0; c < nchunks; ++c) it[c] = dissem::kern::CrcItem{buf + c * chunk, chunk, crc + c};
    CHECK(dissem::kern::crc32c_batch(it, int(nchunks), ws, v0, 0));
    CHECK(hipStreamSynchronize(v0));
    CHECK(hipStreamDestroy(v0));
  }
  std::vector<float> alone;
  rccl_run(lane_all, std::min(secs, 3.0), alone);
  printf("{\"case\": \"rccl_self_p2p_alone\", \"xfer_MiB\": %lld, \"GBps_p50\": %.1f, \"GBps_p10\": %.1f}\n",
         (long long)(xfer >> 20), pct(alone, 0.5), pct(alone, 0.1));
  fflush(stdout);
  struct Case {
    const char* name;
    int cap;
    bool partition;
  };
  const Case cases[] = {{"unmasked_full_grid", 0, false}, {"unmasked_cap32", 32, false}, {"partitioned_last32", 32, true}};
  for (const Case& cs : cases) {
    hipStream_t verify, lane;
    if (cs.partition) {
      verify = make_masked([](int cu, int cus) { return cu >= cus - 32; });
      lane = make_masked([](int cu, int cus) { return cu < cus - 32; });
    } else {
      CHECK(hipStreamCreateWithFlags(&verify, hipStreamNonBlocking));
      lane = make_stream(0, true);
    }
    std::vector<float> alone_here;
    rccl_run(lane, std::min(secs, 3.0), alone_here);
    std::atomic<bool> stop{false};
    std::atomic<int64_t> issued{0};
    std::vector<hipEvent_t> done(kRing);
    for (auto& e : done) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int64_t stalls = 0;
    std::thread th([&] {
      auto next = std::chrono::steady_clock::now();
      for (int64_t b = 0; !stop.load(); ++b) {
        std::this_thread::sleep_until(next);
        next += std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(period_s));
        const int slot = int(b % kRing);
        if (b >= kRing && hipEventQuery(done[size_t(slot)]) == hipErrorNotReady) {
          ++stalls;
          CHECK(hipEventSynchronize(done[size_t(slot)]));
        }
        dissem::kern::CrcItem it[nchunks];
        for (int64_t c = 0; c < nchunks; ++c)
          it[c] = dissem::kern::CrcItem{buf + c * chunk, chunk, crc + slot * nchunks + c};
        CHECK(dissem::kern::crc32c_batch(it, int(nchunks), ws + size_t(slot) * wsb, verify, cs.cap));
        CHECK(hipEventRecord(done[size_t(slot)], verify));
        issued.store(b + 1);
      }
    });
    std::vector<float> beside;
    rccl_run(lane, secs, beside);
    stop.store(true);
    th.join();
    int pending = 0;
    for (auto& e : done)
      if (hipEventQuery(e) == hipErrorNotReady) ++pending;
    CHECK(hipStreamSynchronize(verify));
    printf("{\"case\": \"rccl_self_p2p_beside_verify\", \"layout\": \"%s\", \"land_GBps\": %.0f, \"crc_grid_cap\": %d, "
           "\"GBps_alone_here_p50\": %.1f, \"GBps_p50\": %.1f, \"GBps_p10\": %.1f, \"vs_alone\": %.3f, "
           "\"verified_GBps\": %.1f, \"ring_stalls\": %lld, \"pending_at_end\": %d}\n",
           cs.name, land_gbps, cs.cap, pct(alone_here, 0.5), pct(beside, 0.5), pct(beside, 0.1),
           pct(beside, 0.5) / pct(alone_here, 0.5), double(issued.load()) * double(chunk * nchunks) / secs / 1e9,
           (long long)stalls, pending);
    fflush(stdout);
    for (auto& e : done) CHECK(hipEventDestroy(e));
    CHECK(hipStreamDestroy(verify));
    CHECK(hipStreamDestroy(lane));
  }
  NCHECK(ncclCommDestroy(comm));
  return 0;
}

int main(int argc, char** argv) {
  int trials = 40, reserve = 32;
  double paced_s = 0, land_gbps = 450;
  if (argc > 1 && std::string(argv[1]) == "-cumap") return cumap();
  if (argc > 2 && std::string(argv[1]) == "-rccl") return rccl_paced(atof(argv[2]), argc > 4 ? atof(argv[4]) : 450);
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i];
    if (a == "-trials") trials = atoi(argv[i + 1]);
    else if (a == "-reserve") reserve = atoi(argv[i + 1]);
    else if (a == "-paced") paced_s = atof(argv[i + 1]);
    else if (a == "-gbps") land_gbps = atof(argv[i + 1]);
  }
  if (paced_s > 0) return paced(paced_s, land_gbps, {0, 64, 32, 24, 16});
  CHECK(hipSetDevice(0));
  const int64_t chunk = 64ll << 20, nchunks = 7;
  uint8_t* buf = nullptr;
  CHECK(hipMalloc(&buf, size_t(chunk * nchunks)));
  CHECK(dissem::kern::fill_random(buf, chunk * nchunks, 42, nullptr));
  void* ws = nullptr;
  CHECK(hipMalloc(&ws, dissem::kern::crc32c_batch_workspace_bytes()));
  CHECK(hipMemset(ws, 0, dissem::kern::crc32c_batch_workspace_bytes()));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *crc = nullptr, *probe_out = nullptr;
  CHECK(hipMalloc(&crc, 64 * sizeof(uint32_t)));
  CHECK(hipMalloc(&probe_out, 64 * sizeof(uint32_t)));
  hipStream_t comm;
  CHECK(hipStreamCreateWithFlags(&comm, hipStreamNonBlocking));
  hipEvent_t e0, e1, v0, v1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreate(&v0));
  CHECK(hipEventCreate(&v1));
  const uint64_t ticks = 2000;  // 20 us

  // Probe alone: its own launch + run time.
  std::vector<float> alone;
  for (int t = 0; t < trials; ++t) {
    CHECK(hipEventRecord(e0, comm));
    probe_kernel<<<28, 256, 0, comm>>>(probe_out, ticks);
    CHECK(hipEventRecord(e1, comm));
    CHECK(hipStreamSynchronize(comm));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    alone.push_back(ms * 1e3f);
  }
  auto pct = [](std::vector<float> v, double q) {
    std::sort(v.begin(), v.end());
    return v[size_t(q * double(v.size() - 1))];
  };
  printf("{\"case\": \"probe_alone\", \"p50_us\": %.1f, \"max_us\": %.1f}\n", pct(alone, 0.5), pct(alone, 1.0));

  // The 7 chunks as the engine verifies a landed P2P group: one batched launch
  // on the verify stream, unmasked, masked with the full 256-workgroup grid, and
  // masked with the grid capped at the stream's CUs (what HipBackend does).
  dissem::kern::CrcItem items[nchunks];
  for (int64_t c = 0; c < nchunks; ++c) items[c] = dissem::kern::CrcItem{buf + c * chunk, chunk, crc + c};
  const std::pair<int, int> cases[] = {{0, 0}, {reserve, 0}, {reserve, cus - reserve}};
  for (auto [r, cap] : cases) {
    hipStream_t verify = make_stream(r);
    std::vector<float> lat, burst;
    for (int t = 0; t < trials + 2; ++t) {
      CHECK(hipEventRecord(v0, verify));
      CHECK(dissem::kern::crc32c_batch(items, int(nchunks), ws, verify, cap));
      CHECK(hipEventRecord(v1, verify));
      CHECK(hipEventRecord(e0, comm));
      probe_kernel<<<28, 256, 0, comm>>>(probe_out, ticks);
      CHECK(hipEventRecord(e1, comm));
      CHECK(hipStreamSynchronize(comm));
      CHECK(hipStreamSynchronize(verify));
      float ms = 0, vms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      CHECK(hipEventElapsedTime(&vms, v0, v1));
      if (t >= 2) {  // first trials build the CRC tables
        lat.push_back(ms * 1e3f);
        burst.push_back(vms * 1e3f);
      }
    }
    printf("{\"case\": \"probe_during_7_crc64MiB\", \"reserved_cus\": %d, \"crc_grid_cap\": %d, "
           "\"probe_p50_us\": %.1f, \"probe_p90_us\": %.1f, \"probe_max_us\": %.1f, \"crc_burst_p50_us\": %.1f}\n",
           r, cap, pct(lat, 0.5), pct(lat, 0.9), pct(lat, 1.0), pct(burst, 0.5));
    CHECK(hipStreamDestroy(verify));
  }

  // ---- copy bandwidth beside CRC bursts
  const int64_t copy_bytes = 256ll << 20;  // 4 chunks' worth per copy launch
  uint8_t *csrc = nullptr, *cdst = nullptr;
  CHECK(hipMalloc(&csrc, size_t(copy_bytes)));
  CHECK(hipMalloc(&cdst, size_t(copy_bytes)));
  CHECK(hipMemset(csrc, 1, size_t(copy_bytes)));
  hipStream_t lane = make_stream(0, true);  // all-CU dedicated queue, like a comm lane
  for (int wgs : {32, 64}) {
    const std::pair<int, int> ccases[] = {{-1, 0}, {0, 0}, {reserve, cus - reserve}};  // -1: no CRC
    for (auto [r, cap] : ccases) {
      hipStream_t verify = r >= 0 ? make_stream(r) : nullptr;
      std::vector<float> gbps;
      for (int t = 0; t < trials + 2; ++t) {
        // 3 bursts of 7-chunk CRCs queued ahead, so the copy runs inside them
        if (verify)
          for (int b = 0; b < 3; ++b) CHECK(dissem::kern::crc32c_batch(items, int(nchunks), ws, verify, cap));
        CHECK(hipEventRecord(e0, lane));
        copy_kernel<<<wgs, 256, 0, lane>>>(reinterpret_cast<const uint4*>(csrc), reinterpret_cast<uint4*>(cdst),
                                           copy_bytes / 16);
        CHECK(hipEventRecord(e1, lane));
        CHECK(hipStreamSynchronize(lane));
        if (verify) CHECK(hipStreamSynchronize(verify));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (t >= 2) gbps.push_back(float(double(copy_bytes) / (double(ms) * 1e-3) / 1e9));
      }
      printf("{\"case\": \"copy_beside_crc\", \"copy_workgroups\": %d, \"crc\": %s, \"reserved_cus\": %d, "
             "\"crc_grid_cap\": %d, \"copy_GBps_p50\": %.1f, \"copy_GBps_p10\": %.1f, \"copy_GBps_min\": %.1f}\n",
             wgs, r < 0 ? "false" : "true", r < 0 ? 0 : r, cap, pct(gbps, 0.5), pct(gbps, 0.1), pct(gbps, 0.0));
      if (verify) CHECK(hipStreamDestroy(verify));
    }
  }
  return 0;
}

// ---- continuous verification at the landing rate beside a copy (see the top)
int paced(double secs, double land_gbps, const std::vector<int>& caps) {
  CHECK(hipSetDevice(0));
  const int64_t chunk = 64ll << 20, nchunks = 7;
  uint8_t* buf = nullptr;
  CHECK(hipMalloc(&buf, size_t(chunk * nchunks)));
  CHECK(dissem::kern::fill_random(buf, chunk * nchunks, 42, nullptr));
  const int kRing = 64;  // batches in flight at most (workspace + CRC slots per batch)
  const size_t wsb = dissem::kern::crc32c_batch_workspace_bytes();
  uint8_t* ws = nullptr;
  CHECK(hipMalloc(&ws, wsb * kRing));
  CHECK(hipMemset(ws, 0, wsb * kRing));  // fold words: zeroed once (kernels.h)
  uint32_t* crc = nullptr;
  CHECK(hipMalloc(&crc, size_t(kRing) * nchunks * sizeof(uint32_t)));
  const int64_t copy_bytes = 256ll << 20;
  uint8_t *csrc = nullptr, *cdst = nullptr;
  CHECK(hipMalloc(&csrc, size_t(copy_bytes)));
  CHECK(hipMalloc(&cdst, size_t(copy_bytes)));
  CHECK(hipMemset(csrc, 1, size_t(copy_bytes)));
  hipStream_t lane = make_stream(0, true);
  hipStream_t verify;
  CHECK(hipStreamCreateWithFlags(&verify, hipStreamNonBlocking));
  const double period_s = double(chunk * nchunks) / (land_gbps * 1e9);
  auto copy_run = [&](double dur, std::vector<float>& gbps) {
    const int n = 64;
    std::vector<hipEvent_t> ev(size_t(n) + 1);
    for (auto& e : ev) CHECK(hipEventCreate(&e));
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(dur);
    while (std::chrono::steady_clock::now() < t_end) {
      CHECK(hipEventRecord(ev[0], lane));
      for (int k = 0; k < n; ++k) {
        copy_kernel<<<64, 256, 0, lane>>>(reinterpret_cast<const uint4*>(csrc), reinterpret_cast<uint4*>(cdst),
                                          copy_bytes / 16);
        CHECK(hipEventRecord(ev[size_t(k) + 1], lane));
      }
      CHECK(hipStreamSynchronize(lane));
      for (int k = 0; k < n; ++k) {
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, ev[size_t(k)], ev[size_t(k) + 1]));
        gbps.push_back(float(double(copy_bytes) / (double(ms) * 1e-3) / 1e9));
      }
    }
    for (auto& e : ev) CHECK(hipEventDestroy(e));
  };
  auto pct = [](std::vector<float> v, double q) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.f : v[size_t(q * double(v.size() - 1))];
  };
  std::vector<float> alone;
  copy_run(std::min(secs, 3.0), alone);
  printf("{\"case\": \"paced_copy_alone\", \"copy_workgroups\": 64, \"copy_GBps_p50\": %.1f, \"copy_GBps_p10\": %.1f}\n",
         pct(alone, 0.5), pct(alone, 0.1));
  fflush(stdout);
  // warm the CRC tables
  {
    dissem::kern::CrcItem it[nchunks];
    for (int64_t c = 0; c < nchunks; ++c) it[c] = dissem::kern::CrcItem{buf + c * chunk, chunk, crc + c};
    CHECK(dissem::kern::crc32c_batch(it, int(nchunks), ws, verify, 0));
    CHECK(hipStreamSynchronize(verify));
  }
  for (int cap : caps) {
    std::atomic<bool> stop{false};
    std::atomic<int64_t> issued{0};
    std::vector<hipEvent_t> done(kRing);
    for (auto& e : done) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int64_t stalls = 0;  // ring full: the verify fell a whole ring behind
    std::thread th([&] {
      auto next = std::chrono::steady_clock::now();
      for (int64_t b = 0; !stop.load(); ++b) {
        std::this_thread::sleep_until(next);
        next += std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(period_s));
        const int slot = int(b % kRing);
        if (b >= kRing && hipEventQuery(done[size_t(slot)]) == hipErrorNotReady) {
          ++stalls;
          CHECK(hipEventSynchronize(done[size_t(slot)]));
        }
        dissem::kern::CrcItem it[nchunks];
        for (int64_t c = 0; c < nchunks; ++c)
          it[c] = dissem::kern::CrcItem{buf + c * chunk, chunk, crc + slot * nchunks + c};
        CHECK(dissem::kern::crc32c_batch(it, int(nchunks), ws + size_t(slot) * wsb, verify, cap));
        CHECK(hipEventRecord(done[size_t(slot)], verify));
        issued.store(b + 1);
      }
    });
    std::vector<float> beside;
    copy_run(secs, beside);
    stop.store(true);
    th.join();
    // still pending at the end, and the time the verify stream needs to drain
    int pending = 0;
    for (auto& e : done)
      if (hipEventQuery(e) == hipErrorNotReady) ++pending;
    const auto d0 = std::chrono::steady_clock::now();
    CHECK(hipStreamSynchronize(verify));
    const double drain_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d0).count();
    const double verified_gbps = double(issued.load()) * double(chunk * nchunks) / secs / 1e9;
    printf("{\"case\": \"paced_copy_beside_verify\", \"land_GBps\": %.0f, \"crc_grid_cap\": %d, \"copy_workgroups\": 64, "
           "\"copy_GBps_p50\": %.1f, \"copy_GBps_p10\": %.1f, \"copy_vs_alone\": %.3f, \"verified_GBps\": %.1f, "
           "\"batches\": %lld, \"ring_stalls\": %lld, \"pending_at_end\": %d, \"drain_ms\": %.2f}\n",
           land_gbps, cap, pct(beside, 0.5), pct(beside, 0.1), pct(beside, 0.5) / pct(alone, 0.5), verified_gbps,
           (long long)issued.load(), (long long)stalls, pending, drain_ms);
    fflush(stdout);
    for (auto& e : done) CHECK(hipEventDestroy(e));
  }
  // CU partitions: the verify stream on a set of CUs (grid = that many
  // workgroups, one per CU), the copy lane on the rest - no workgroup of one
  // ever shares a CU with the other. Sets: the last 32 mask bits
  // (contiguous), every 8th bit (32 CUs spread over the mask), every 4th (64).
  struct Part {
    const char* name;
    int every, phase, n;  // every < 0: contiguous last n
  };
  const Part parts[] = {{"last32", -1, 0, 32}, {"every8th", 8, 7, 32}, {"every4th", 4, 3, 64}};
  for (const Part& pt : parts) {
    auto is_verify = [pt](int cu, int cus) { return pt.every < 0 ? cu >= cus - pt.n : cu % pt.every == pt.phase; };
    hipStream_t vs = make_masked([&](int cu, int cus) { return is_verify(cu, cus); });
    hipStream_t ls = make_masked([&](int cu, int cus) { return !is_verify(cu, cus); });
    std::swap(verify, vs);
    std::swap(lane, ls);
    std::vector<float> alone_p;
    copy_run(std::min(secs, 3.0), alone_p);
    std::atomic<bool> stop{false};
    std::atomic<int64_t> issued{0};
    std::vector<hipEvent_t> done(kRing);
    for (auto& e : done) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int64_t stalls = 0;
    std::thread th([&] {
      auto next = std::chrono::steady_clock::now();
      for (int64_t b = 0; !stop.load(); ++b) {
        std::this_thread::sleep_until(next);
        next += std::chrono::duration_cast<std::chrono::steady_clock::duration>(std::chrono::duration<double>(period_s));
        const int slot = int(b % kRing);
        if (b >= kRing && hipEventQuery(done[size_t(slot)]) == hipErrorNotReady) {
          ++stalls;
          CHECK(hipEventSynchronize(done[size_t(slot)]));
        }
        dissem::kern::CrcItem it[nchunks];
        for (int64_t c = 0; c < nchunks; ++c)
          it[c] = dissem::kern::CrcItem{buf + c * chunk, chunk, crc + slot * nchunks + c};
        CHECK(dissem::kern::crc32c_batch(it, int(nchunks), ws + size_t(slot) * wsb, verify, pt.n));
        CHECK(hipEventRecord(done[size_t(slot)], verify));
        issued.store(b + 1);
      }
    });
    std::vector<float> beside;
    copy_run(secs, beside);
    stop.store(true);
    th.join();
    int pending = 0;
    for (auto& e : done)
      if (hipEventQuery(e) == hipErrorNotReady) ++pending;
    const auto d0 = std::chrono::steady_clock::now();
    CHECK(hipStreamSynchronize(verify));
    const double drain_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d0).count();
    printf("{\"case\": \"paced_partitioned\", \"land_GBps\": %.0f, \"verify_cus\": \"%s\", \"crc_grid_cap\": %d, "
           "\"copy_GBps_alone_p50\": %.1f, \"copy_GBps_p50\": %.1f, \"copy_GBps_p10\": %.1f, \"copy_vs_alone\": %.3f, "
           "\"copy_vs_all_cu_alone\": %.3f, \"verified_GBps\": %.1f, \"ring_stalls\": %lld, \"pending_at_end\": %d, "
           "\"drain_ms\": %.2f}\n",
           land_gbps, pt.name, pt.n, pct(alone_p, 0.5), pct(beside, 0.5), pct(beside, 0.1),
           pct(beside, 0.5) / pct(alone_p, 0.5), pct(beside, 0.5) / pct(alone, 0.5),
           double(issued.load()) * double(chunk * nchunks) / secs / 1e9, (long long)stalls, pending, drain_ms);
    fflush(stdout);
    for (auto& e : done) CHECK(hipEventDestroy(e));
    std::swap(verify, vs);
    std::swap(lane, ls);
    CHECK(hipStreamDestroy(vs));
    CHECK(hipStreamDestroy(ls));
  }
  return 0;
}
