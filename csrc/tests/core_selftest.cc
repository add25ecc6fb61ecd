// Host-only self test of the native core, built under ThreadSanitizer and
// AddressSanitizer (`make sanitize`). Exercises the concurrent
// paths: TCP + in-proc transports, every role/mode on the host engine, and the
// planned (GPU-schedule) engine on the simulated RCCL fabric with 4 ranks.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>

#include "core/crc32c.h"
#include "core/vclock.h"
#include "core/log.h"
#include "engine/planned_engine.h"
#include "roles/node.h"

using namespace dissem;

static int failures = 0;
#define EXPECT(c)                                                    \
  do {                                                               \
    if (!(c)) {                                                      \
      fprintf(stderr, "FAILED %s at %s:%d\n", #c, __FILE__, __LINE__); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

static std::shared_ptr<HostBuffer> random_buf(int64_t n, uint32_t seed) {
  auto b = HostBuffer::alloc(n, false);
  std::mt19937 rng(seed);
  for (int64_t i = 0; i < n; ++i) b->ptr[i] = uint8_t(rng());
  return b;
}

static LayerSrc inmem(std::shared_ptr<HostBuffer> b) {
  LayerSrc s;
  s.host = b;
  s.data_size = b->size;
  s.meta = LayerMeta{Location::Inmem, 0, SourceType::Mem, b->size};
  return s;
}

// Ring fixture (node_test.go:45-72) on host engines, all modes, one transport kind.
static void ring(bool tcp, int mode) {
  const int n = 4;
  const int64_t size = (1 << 18) + 13;
  std::vector<std::shared_ptr<Transport>> ts;
  AddrRegistry reg;
  static int uniq = 0;
  ++uniq;
  for (int i = 0; i <= n; ++i) {
    if (tcp) {
      ts.push_back(make_tcp_transport("127.0.0.1:0", {}));
      reg[NodeID(i)] = ts.back()->address();
    } else {
      reg[NodeID(i)] = "r" + std::to_string(uniq) + "-" + std::to_string(i);
    }
  }
  if (!tcp)
    for (int i = 0; i <= n; ++i) ts.push_back(make_inproc_transport(reg[NodeID(i)], reg));
  for (auto& t : ts) t->set_registry(reg);
  LayersSrc all;
  Assignment asg;
  for (int i = 1; i <= n; ++i) {
    all[LayerID(i)] = inmem(random_buf(size, uint32_t(i)));
    asg[NodeID(i)][LayerID(i)] = LayerMeta{};
  }
  std::vector<std::unique_ptr<Node>> nodes;
  NodeConfig lc;
  lc.id = 0;
  lc.leader = 0;
  lc.mode = mode;
  nodes.push_back(std::make_unique<Node>(lc, ts[0], make_host_engine(), all, asg, true));
  for (int i = 1; i <= n; ++i) {
    NodeConfig c;
    c.id = NodeID(i);
    c.leader = 0;
    c.mode = mode;
    LayersSrc mine;
    if (mode > 0) {
      int prev = ((i - 2 + n) % n) + 1;
      mine[LayerID(prev)] = all[LayerID(prev)];
    }
    nodes.push_back(std::make_unique<Node>(c, ts[size_t(i)], make_host_engine(), mine, Assignment{}, false));
  }
  for (auto& nd : nodes) nd->start();
  for (size_t i = 1; i < nodes.size(); ++i) nodes[i]->announce();
  EXPECT(nodes[0]->wait_ready(10));
  for (size_t i = 1; i < nodes.size(); ++i) {
    EXPECT(nodes[i]->wait_ready(10));
    LayerSrc got;
    EXPECT(nodes[i]->store().get(LayerID(i), &got));
    EXPECT(got.host && memcmp(got.host->ptr, all[LayerID(i)].host->ptr, size_t(size)) == 0);
  }
  for (auto& nd : nodes) nd->stop();
  nodes.clear();
  for (auto& t : ts) t->close();
}

// Planned engine on the simulated fabric: 4 ranks, full replication.
// die >= 0: that rank stops dead after two groups (elastic recovery path;
// every layer then has two holders). crossing: two holders per layer and
// mode-2 chunk jobs: steals move jobs between the holders, never a dest's own
// load of a layer it holds (that would write its chunks twice: the race TSAN
// found here in round 5).
// virt: on the virtual clock with modeled link and staging rates (the
// simulator's model-time mode, scripts/predict_scaling.py): every engine,
// node and fabric thread waits through vclock, the main thread uncounted.
static void planned_sim(int mode, double corrupt = 0, int die = -1, bool crossing = false, bool virt = false) {
  const int n = 4, L = 6;
  const int64_t chunk = 1 << 16, size = 3 * chunk + 100;
  static int uniq = 0;
  std::string key = "tsan" + std::to_string(++uniq);
  if (virt) {
    vclock::enable(true);
    SimTiming t;
    t.link_bps = 1e9;   // 64 KiB chunks: 65 us per transfer in model time
    t.stage_bps = 2e9;
    t.verify_bps = 50e9;
    t.verify_launch_s = 10e-6;
    sim_set_timing(key, t);
  }
  AddrRegistry reg;
  for (int i = 0; i < n; ++i) reg[NodeID(i)] = key + "-" + std::to_string(i);
  std::vector<std::shared_ptr<Transport>> ts;
  for (int i = 0; i < n; ++i) ts.push_back(make_inproc_transport(reg[NodeID(i)], reg));
  std::vector<std::shared_ptr<PlannedEngine>> engines;
  std::vector<std::shared_ptr<HostBuffer>> data;
  for (int l = 0; l < L; ++l) data.push_back(random_buf(size, uint32_t(100 + l)));
  Assignment asg;
  for (int i = 0; i < n; ++i)
    for (int l = 0; l < L; ++l) asg[NodeID(i)][LayerID(l)] = LayerMeta{};
  std::vector<std::unique_ptr<Node>> nodes;
  for (int i = 0; i < n; ++i) {
    PlannedConfig pc;
    pc.rank = i;
    pc.world = n;
    pc.chunk_bytes = chunk;
    pc.inject_corrupt = corrupt;
    pc.max_retries = 16;
    if (die >= 0) {
      pc.suspect_s = 0.2;
      if (i == die) pc.inject_die_after_groups = 2;
    }
    auto e = std::make_shared<PlannedEngine>(pc, make_sim_backend(key, i, n, resolve_lanes(pc)));  // directed lanes
    LayersSrc mine;
    for (int l = 0; l < L; ++l) {
      e->provision(LayerID(l), size);
      if (l % n == i || ((die >= 0 || crossing) && (l + 1) % n == i)) {
        mine[LayerID(l)] = inmem(data[size_t(l)]);
        CrcManifest m;
        m.chunk_bytes = chunk;
        for (int64_t off = 0; off < size; off += chunk)
          m.crc.push_back(crc32c_raw(data[size_t(l)]->ptr + off, size_t(std::min(chunk, size - off)), 0xFFFFFFFFu) ^
                          0xFFFFFFFFu);
        e->set_manifest(LayerID(l), m);
      }
    }
    if (getenv("SELFTEST_PTRS"))
      for (int l = 0; l < L; ++l) fprintf(stderr, "rank %d layer %d slot %p\n", i, l, (void*)e->device_ptr(LayerID(l)));
    engines.push_back(e);
    NodeConfig c;
    c.id = NodeID(i);
    c.leader = 0;
    c.mode = mode;
    c.pull_window = 3;
    if (crossing) {
      c.pull_job_bytes = chunk;
      c.range_acks = true;
    }
    nodes.push_back(std::make_unique<Node>(c, ts[size_t(i)], e, mine, i == 0 ? asg : Assignment{}, i == 0));
  }
  for (auto& nd : nodes) nd->start();
  for (int i = 1; i < n; ++i) nodes[size_t(i)]->announce();
  for (int i = 0; i < n; ++i)
    if (i != die) EXPECT(nodes[size_t(i)]->wait_ready(20));
  if (die >= 0) EXPECT(nodes[0]->stats().recoveries == 1);
  for (int i = 0; i < n; ++i) {
    if (i == die) continue;
    engines[size_t(i)]->quiesce();
    for (int l = 0; l < L; ++l)
      EXPECT(memcmp(engines[size_t(i)]->device_ptr(LayerID(l)), data[size_t(l)]->ptr, size_t(size)) == 0);
    EXPECT(engines[size_t(i)]->error().empty());
    EXPECT(engines[size_t(i)]->stats().order_violations == 0);
  }
  for (auto& nd : nodes) nd->stop();
  nodes.clear();
  for (auto& e : engines) e->shutdown();
  for (auto& t : ts) t->close();
  if (virt) {
    EXPECT(vclock::now() > 0);
    vclock::enable(false);
  }
}

int main(int argc, char** argv) {
  log::set_level(log::Error);
  // optional: run one case only (0-3 ring modes, 4-6 planned modes 1-3, 7 corruption, 8-9 rank death,
  // 10 crossing mode-2 chunk jobs, 11-13 planned modes 1-3 on the virtual clock)
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  auto on = [&](int k) { return only < 0 || only == k; };
  for (int mode = 0; mode <= 3; ++mode) {
    if (!on(mode)) continue;
    ring(false, mode);
    ring(true, mode);
  }
  for (int mode = 1; mode <= 3; ++mode)
    if (on(3 + mode)) planned_sim(mode);
  if (on(7)) planned_sim(1, 0.3);  // NACK / re-send path under injected corruption
  if (on(8)) planned_sim(1, 0, 3);  // a rank dies: suspect -> probe -> shrink -> re-plan
  if (on(9)) planned_sim(2, 0, 2);
  if (on(10)) planned_sim(2, 0, -1, true);
  for (int mode = 1; mode <= 3; ++mode)
    if (on(10 + mode)) planned_sim(mode, 0, -1, mode == 2, true);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("core selftest ok\n");
  return 0;
}
